"""Summarise a rocprofv3 kernel_trace.csv: per (kernel, grid) totals and per family.
usage: python scripts/kt_summary.py kernel_trace.csv [batches] [ledger.txt steps]
With a step ledger (scripts/ledger.py) and the DDIM steps per batch, each MFMA family's trace time is
set against the ledger's algorithmic FLOP: fraction of the 2.5 PF/s dense peak, time-weighted over
the family's kernels in the trace (the igemm family = 3x3 + 1x1 + GEGLU + the split-K combine)."""
import collections
import csv
import sys

path = sys.argv[1]
nb = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
agg = collections.defaultdict(lambda: [0, 0.0])
fam = collections.defaultdict(float)


def _ks(n):
    """KS template argument (1 = 1x1 GEMM, 3 = 3x3 conv) of the implicit-GEMM kernels."""
    args = [a.strip() for a in n[n.index("<") + 1:n.index(">")].split(",")]
    if "igemm_pp16_kernel" in n:
        return args[1]
    if "igemm_m32_kernel" in n:
        return args[6]
    return args[-1]


def family(n):
    if "igemm_pp16r_kernel" in n:   # the row-ring tile is 3x3-only (its template has no KS argument)
        return "conv3x3"
    if "igemm_" in n and "<" in n and "igemm_kernel" not in n:
        return "conv3x3" if _ks(n) == "3" else "gemm1x1"
    for key, f in (("igemm_kernel", "gemm_reg"), ("splitk", "splitk"), ("attn_fwd", "attention"), ("attn_small", "attention"),
                   ("window_attn", "attention"), ("gn_", "groupnorm"), ("ln_", "layernorm"),
                   ("upsample", "upsample"), ("softmax", "softmax"), ("mel", "logmel")):
        if key in n:
            return f
    return "other"


for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    g = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[(n[:110], g)][0] += 1
    agg[(n[:110], g)][1] += d
    fam[family(n)] += d
tot = sum(v[1] for v in agg.values())
# device idle between consecutive kernels (gaps under 100 us: launch / graph-node overhead,
# not host pauses between phases)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path)))
gap = 0.0
end = iv[0][1] if iv else 0
for a, b in iv[1:]:
    if a > end and a - end < 100_000:
        gap += (a - end) / 1e3
    end = max(end, b)
print(f"device idle between kernels (gaps < 100 us): {gap / 1e3 / nb:.1f} ms per batch")
print(f"total {tot / 1e3:.1f} ms kernel time ({tot / 1e3 / nb:.1f} ms per batch over {nb:g} batches)")
for f, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"  {f:10s} {v / 1e3 / nb:8.1f} ms/batch {100 * v / tot:5.1f}%")
if len(sys.argv) > 4:
    led, steps = {}, float(sys.argv[4])
    for line in open(sys.argv[3]):
        f = line.split()
        if len(f) == 9 and f[0] in ("igemm", "conv3x3", "gemm1x1", "geglu", "attention"):
            led[f[0]] = float(f[4]) * 1e9   # GFLOP per step
    tr = {"conv3x3": fam["conv3x3"], "gemm1x1+geglu": fam["gemm1x1"], "attention": fam["attention"],
          "igemm": fam["conv3x3"] + fam["gemm1x1"] + fam["splitk"] + fam["gemm_reg"]}
    fl = {"conv3x3": led.get("conv3x3", 0), "gemm1x1+geglu": led.get("gemm1x1", 0) + led.get("geglu", 0),
          "attention": led.get("attention", 0), "igemm": led.get("igemm", 0)}
    print(f"family MFMA fraction over the trace (ledger FLOP x {steps:g} steps per batch / trace time per batch):")
    for f in ("igemm", "conv3x3", "gemm1x1+geglu", "attention"):
        t = tr[f] / 1e6 / nb   # seconds per batch
        if t > 0:
            print(f"  {f:14s} {fl[f] * steps / 1e12:8.1f} TFLOP / {t * 1e3:7.1f} ms = {fl[f] * steps / t / 2.5e15:.3f}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:70]:
    print(f"{v[1] / 1e3:9.2f} ms {100 * v[1] / tot:5.1f}% {v[0]:6d} {v[1] / v[0]:9.1f}us grid={k[1]} {k[0]}")
