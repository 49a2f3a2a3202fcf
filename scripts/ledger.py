"""Per-shape roofline ledger of one CFG+DDIM denoise step (the GraphDenoiser body).

Records every c2d op the UNet step issues (ops.conv / attention / group_norm[_stats|_apply] /
layer_norm[_stats] / add / upsample_nearest2x) during one eager step, groups the calls by
signature, and times each unique call as a hipGraph of `reps` back-to-back launches on the
recorded tensors (HIP events on the capture's stream, min over replays).  Every row carries its
algorithmic work and its binding roof:

  conv / GEMM   FLOP = 2 * M_out * N * k^2 * C_in         (N = packed GEGLU width for GEGLU)
                bytes = source (+ second source) + weights + output (+ residual), fp16
  attention     FLOP = 4 * (batch * heads) * Lq * Lk * d     bytes = q + k + v + o, fp16
  norms / add / upsample: bytes = one read of every input + one write of every output
  roof_us = max(FLOP / 2.5 PF/s, bytes / 8 TB/s);  frac = roof_us / us;  lost = calls * (us - roof_us)

The step itself is replayed as its captured graph and timed too: its time minus the sum of the
rows is what the ledger does not attribute (torch copies, launch gaps, cross-op cache effects).

  python scripts/ledger.py --batch 8 [--res 64] [--reps 10] [--out profiles/r05_ledger_c3.txt]
  python scripts/ledger.py --vae --batch 8 --res 64     (one VAE decode of 8 latents instead)
bench.py imports `step_ledger` for roofline.family_frac.
"""
from __future__ import annotations

import argparse
import collections
import inspect
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

PEAK_FLOPS = 2.5e15    # dense fp16 MFMA (MI355X_MICROARCH.md)
PEAK_BYTES = 8.0e12    # HBM3E
RECORDED = ("conv", "attention", "group_norm", "group_norm_stats", "group_norm_apply", "layer_norm",
            "layer_norm_stats", "add", "upsample_nearest2x")


def _nb(t) -> int:
    return 0 if t is None else t.numel() * t.element_size()


def _rows(t) -> int:
    return t.numel() // t.shape[-1]


def _sig(v):
    if torch.is_tensor(v):
        return ("T", tuple(v.shape), tuple(v.stride()), str(v.dtype))
    if isinstance(v, (tuple, list)):
        return tuple(_sig(u) for u in v)
    if isinstance(v, dict):
        return tuple(sorted((k, _sig(u)) for k, u in v.items()))
    return v


def _work(name: str, a: dict, out) -> tuple[str, str, float, float]:
    """(family, description, FLOP, bytes) of one recorded call (bound arguments `a`)."""
    if name == "conv":
        x, x2, k = a["x"], a["x2"], a["ksize"]
        cin = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
        cout = a["cout"]
        m = _rows(out)
        flop = 2.0 * m * cout * k * k * cin
        byts = _nb(x) + _nb(x2) + cout * k * k * cin * 2 + _nb(out) + (m * out.shape[-1] * 2 if a["resid"] is not None else 0)
        act = a["act"]
        fam = "geglu" if act == "geglu" else ("conv3x3" if k == 3 else "gemm1x1")
        desc = (f"{'3x3' if k == 3 else '1x1'} M={m} {cin}->{cout}" + (f" s{a['stride']}" if a["stride"] > 1 else "")
                + (" up" if a["up"] else "") + (" pad" if a["padded"] else "") + (f" {act}" if act else "")
                + (" +gn" if a["gn"] is not None else "") + (" +ln" if a["ln"] is not None else "")
                + (" +res" if a["resid"] is not None else "") + (" +temb" if a["temb"] is not None else "")
                + (" +gnm" if a.get("gn_moments") else ""))
        return fam, desc, flop, byts
    if name == "attention":
        bh, lq, lk, d = a["batch"] * a["heads"], a["lq"], a["lk"], a["d"]
        flop = 4.0 * bh * lq * lk * d
        byts = 2.0 * (2 * bh * lq * d + 2 * bh * lk * d)
        kb = a["key_bias"]
        desc = f"b*h={bh} lq={lq} lk={lk} d={d}" + (" +bias" if kb is not None else "")
        return "attention", desc, flop, byts
    if name in ("group_norm", "group_norm_apply", "group_norm_stats"):
        x, x2 = a["x"], a["x2"]
        byts = _nb(x) + _nb(x2) + (_nb(out) if name != "group_norm_stats" else 0)
        flag = {"group_norm": " pad" if a.get("pad") else "", "group_norm_stats": " stats",
                "group_norm_apply": " apply"}[name]
        silu = (" silu" if a.get("silu") else "") + (" mom" if a.get("mom") is not None else "")
        c = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
        return "groupnorm", f"GN {tuple(x.shape[:-1])}x{c}{flag}{silu}", 0.0, float(byts)
    if name in ("layer_norm", "layer_norm_stats"):
        x = a["x2d"]
        byts = _nb(x) + (_nb(out) if name == "layer_norm" else 0)
        return "layernorm", f"LN {tuple(x.shape)}" + (" stats" if name.endswith("stats") else ""), 0.0, float(byts)
    if name == "add":
        return "elementwise", f"add {tuple(a['a'].shape)}", 0.0, float(3 * _nb(a["a"]))
    if name == "upsample_nearest2x":
        return "elementwise", f"upsample2x {tuple(a['x'].shape)}", 0.0, float(_nb(a["x"]) + _nb(out))
    raise KeyError(name)


class Recorder:
    """Patches the recorded ops (ops module attribute and any clap2diffusion_amd module that
    imported them by name) for the duration of a `with` block."""

    def __init__(self):
        self.calls = []
        self.orig = {n: getattr(ops, n) for n in RECORDED}

    def _wrap(self, name):
        fn = self.orig[name]
        sig = inspect.signature(fn)

        def rec(*args, **kw):
            res = fn(*args, **kw)
            b = sig.bind(*args, **kw)
            b.apply_defaults()
            # conv(..., gn_moments=G) returns (out, moments): the row accounts the output tensor
            self.calls.append((name, b, res[0] if isinstance(res, tuple) else res))
            return res
        return rec

    def __enter__(self):
        self.patched = []
        wraps = {n: self._wrap(n) for n in RECORDED}
        for mod in list(sys.modules.values()):
            if mod is None or not getattr(mod, "__name__", "").startswith("clap2diffusion_amd"):
                continue
            for n in RECORDED:
                if getattr(mod, n, None) is self.orig[n]:
                    setattr(mod, n, wraps[n])
                    self.patched.append((mod, n))
        return self

    def __exit__(self, *exc):
        for mod, n in self.patched:
            setattr(mod, n, self.orig[n])
        return False


def _time_graph(fn, reps: int, tries: int = 3) -> float:
    """us per call of fn(), captured `reps` times into one graph (min over `tries` replays)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = math.inf
    for _ in range(tries):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def _call_kwargs(b, out) -> dict:
    kw = dict(b.arguments)
    if "out" in kw and kw["out"] is None and torch.is_tensor(out):
        kw["out"] = out
    return kw


def in_situ(rec, rows, top: int = 3, tries: int = 3):
    """In-situ times of the families and of the `top` heaviest signatures of a recorded call
    sequence: the whole sequence (every recorded call, in its recorded order, on its recorded
    tensors) is captured as ONE graph and timed, then once more per family / signature with that
    family's / signature's calls left out; a family's in-situ time is the difference.  Unlike the
    10x back-to-back replays of the rows (each call's weights hot in L2 / MALL, the clock of a
    repeated kernel), every call here runs after its real predecessor, as in the step.
    -> (sequence us, {family: us}, [(row, us)])"""
    calls = []
    for name, b, out in rec.calls:
        fam = _work(name, b.arguments, out)[0]
        calls.append((rec.orig[name], _call_kwargs(b, out), fam, (name, _sig(dict(b.arguments)))))

    def seq_us(skip) -> float:
        kept = [(fn, kw) for fn, kw, fam, sg in calls if not skip(fam, sg)]

        def run():
            for fn, kw in kept:
                fn(**kw)
        return _time_graph(run, 1, tries)

    with torch.no_grad():
        whole = seq_us(lambda fam, sg: False)
        fam_us = {}
        for fam in dict.fromkeys(c[2] for c in calls):
            fam_us[fam] = whole - seq_us(lambda f, sg, fam=fam: f == fam)
        heavy = sorted(rows, key=lambda r: -r["calls"] * r["us"])[:top]
        sig_us = [(r, whole - seq_us(lambda f, sg, key=r["key"]: sg == key)) for r in heavy]
    return whole, fam_us, sig_us


def call_ledger(run, reps: int = 10, keep_recording: bool = False):
    """Ledger of the c2d calls one invocation of run() issues; -> (rows, families, n_calls)
    (keep_recording: and the Recorder, for in_situ)."""
    rec = Recorder()
    with torch.no_grad(), rec:
        run()
    torch.cuda.synchronize()
    groups = collections.OrderedDict()
    for name, b, out in rec.calls:
        groups.setdefault((name, _sig(dict(b.arguments))), []).append((b, out))
    rows = []
    with torch.no_grad():
        for key, lst in groups.items():
            name = key[0]
            b, out = lst[0]
            kw = _call_kwargs(b, out)
            fn = rec.orig[name]
            plan = None
            if name == "conv":
                with ops.record_conv_plans() as plans:
                    fn(**kw)
                plan = plans[0] if plans else None
            us = _time_graph(lambda: fn(**kw), reps)
            fam, desc, flop, byts = _work(name, b.arguments, out)
            roof_us = max(flop / PEAK_FLOPS, byts / PEAK_BYTES) * 1e6
            bound = "mfma" if flop / PEAK_FLOPS >= byts / PEAK_BYTES else "hbm"
            rows.append(dict(op=name, key=key, family=fam, desc=desc, calls=len(lst), plan=plan, us=us, flop=flop,
                             bytes=byts, roof_us=roof_us, bound=bound, frac=roof_us / us,
                             lost_us=len(lst) * (us - roof_us)))
    rows.sort(key=lambda r: -r["lost_us"])
    fams = collections.OrderedDict()
    for r in rows:
        for f in (r["family"], "igemm" if r["op"] == "conv" else None, "all"):
            if f is None:
                continue
            s_ = fams.setdefault(f, dict(calls=0, us=0.0, flop=0.0, bytes=0.0, roof_us=0.0))
            s_["calls"] += r["calls"]
            s_["us"] += r["calls"] * r["us"]
            s_["flop"] += r["calls"] * r["flop"]
            s_["bytes"] += r["calls"] * r["bytes"]
            s_["roof_us"] += r["calls"] * r["roof_us"]
    for s_ in fams.values():
        s_["frac"] = s_["roof_us"] / s_["us"] if s_["us"] else 0.0
        s_["mfma_frac"] = s_["flop"] / (s_["us"] * 1e-6) / PEAK_FLOPS if s_["us"] else 0.0
    if keep_recording:
        return rows, fams, len(rec.calls), rec
    return rows, fams, len(rec.calls)


def step_ledger(den, reps: int = 10, situ: bool = False):
    """Ledger of one step of a GraphDenoiser `den` (its eager body); -> (rows, families, meta).
    rows: dicts sorted by lost us per step.  The denoiser's step counter is restored.
    situ: also the in-situ family / heaviest-signature times (in_situ) in meta["in_situ"]."""
    idx0 = den.step_idx.clone()
    den.step_idx.zero_()
    rows, fams, ncalls, rec = call_ledger(den._body, reps, keep_recording=True)
    situ_meta = None
    if situ:
        whole, fam_us, sig_us = in_situ(rec, rows)
        situ_meta = dict(sequence_us=whole, family_us=fam_us, heavy=sig_us)
    step_us = None
    if den.graph is not None:
        ts = []
        for _ in range(3):
            den.step_idx.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            den.graph.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        step_us = min(ts)
    den.step_idx.copy_(idx0)
    meta = dict(n_calls=ncalls, unique=len(rows), step_us=step_us, n=2 * den.b, res=den.h, what="denoise step",
                in_situ=situ_meta)
    return rows, fams, meta


def vae_ledger(vae, latents, reps: int = 5):
    """Ledger of one VAE decode of `latents` [B, 4, h, w]; the whole decode timed as a graph too."""
    rows, fams, ncalls = call_ledger(lambda: vae(latents), reps)
    whole = _time_graph(lambda: vae(latents), 1)
    meta = dict(n_calls=ncalls, unique=len(rows), step_us=whole, n=latents.shape[0], res=latents.shape[-1],
                what="VAE decode")
    return rows, fams, meta


def format_ledger(rows, fams, meta) -> str:
    tot = fams["all"]["us"]
    what = meta.get("what", "denoise step")
    head = (f"N = {meta['n']} (CFG pair x {meta['n'] // 2})" if what == "denoise step" else f"B = {meta['n']}")
    L = [f"# {what} ledger: {head}, {meta['res']}^2 latent; "
         f"{meta['n_calls']} recorded c2d calls, {meta['unique']} unique signatures",
         f"# sum of rows {tot / 1e3:.3f} ms per {what}" + (
             f"; captured graph {meta['step_us'] / 1e3:.3f} ms (unattributed {(meta['step_us'] - tot) / 1e3:.3f} ms)"
             if meta["step_us"] else ""),
         "# roofs: 2.5 PF/s dense fp16 MFMA, 8 TB/s HBM; frac = roof_us / us; lost = calls x (us - roof_us)",
         "",
         f"{'family':12s} {'calls':>5s} {'ms/step':>8s} {'share':>6s} {'GFLOP':>9s} {'MB':>9s} {'roof ms':>8s} "
         f"{'frac':>6s} {'mfma':>6s}"]
    for f, s in sorted(fams.items(), key=lambda kv: -kv[1]["us"]):
        L.append(f"{f:12s} {s['calls']:5d} {s['us'] / 1e3:8.3f} {100 * s['us'] / tot:5.1f}% {s['flop'] / 1e9:9.1f} "
                 f"{s['bytes'] / 1e6:9.1f} {s['roof_us'] / 1e3:8.3f} {s['frac']:6.3f} {s['mfma_frac']:6.3f}")
    si = meta.get("in_situ")
    if si:
        L += ["", f"# in situ (the recorded call sequence as one graph, {si['sequence_us'] / 1e3:.3f} ms; a family's "
                  "time = sequence - sequence without it)",
              f"{'family':12s} {'ms/step':>8s} {'share':>6s} {'frac':>6s}"]
        for f, us in sorted(si["family_us"].items(), key=lambda kv: -kv[1]):
            s_ = fams[f]
            work = s_["flop"] / PEAK_FLOPS if s_["flop"] > 0 else s_["bytes"] / PEAK_BYTES
            L.append(f"{f:12s} {us / 1e3:8.3f} {100 * us / si['sequence_us']:5.1f}% {work * 1e6 / us if us > 0 else 0:6.3f}")
        for r, us in si["heavy"]:
            work = r["flop"] / PEAK_FLOPS if r["flop"] > 0 else r["bytes"] / PEAK_BYTES
            L.append(f"  heavy: {r['family']}: {r['desc']} x{r['calls']}: {us / 1e3:.3f} ms in situ "
                     f"({us / r['calls']:.1f} us/call, frac {r['calls'] * work * 1e6 / us if us > 0 else 0:.3f}; "
                     f"isolated {r['us']:.1f} us/call)")
    L += ["", f"{'lost us':>8s} {'calls':>5s} {'us/call':>8s} {'roof us':>8s} {'bound':>5s} {'frac':>6s} "
              f"{'GFLOP':>8s} {'MB':>8s} {'plan':>8s}  family / shape"]
    for r in rows:
        pl = f"{r['plan'][0]}/{r['plan'][1]}" if r["plan"] else "-"
        L.append(f"{r['lost_us']:8.1f} {r['calls']:5d} {r['us']:8.1f} {r['roof_us']:8.1f} {r['bound']:>5s} "
                 f"{r['frac']:6.3f} {r['flop'] / 1e9:8.2f} {r['bytes'] / 1e6:8.2f} {pl:>8s}  {r['family']}: {r['desc']}")
    return "\n".join(L) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--res", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--vae", action="store_true", help="ledger of one VAE decode of B latents instead")
    a = ap.parse_args()
    if a.vae:
        from clap2diffusion_amd.vae import VAEDecoder
        from clap2diffusion_amd.weights import synth_vae_decoder
        dev = torch.device("cuda")
        vae = VAEDecoder().to(dev)
        vae.load_diffusers_state_dict(synth_vae_decoder(0))
        lat = torch.randn(a.batch, 4, a.res, a.res, generator=torch.Generator().manual_seed(0)).to(dev)
        with torch.no_grad():
            vae(lat)
        torch.cuda.synchronize()
        txt = format_ledger(*vae_ledger(vae, lat, a.reps))
        print(txt, flush=True)
        if a.out:
            Path(a.out).write_text(txt)
        return
    from clap2diffusion_amd.processor import AudioProcessorManager
    from clap2diffusion_amd.sampler import GraphDenoiser
    from clap2diffusion_amd.scheduler import DDIMScheduler
    from clap2diffusion_amd.unet import UNet2DConditionModel
    from clap2diffusion_amd.weights import synth_unet
    dev = torch.device("cuda")
    unet = UNet2DConditionModel().to(dev)
    unet.load_diffusers_state_dict(synth_unet(0, device=dev))
    mgr = AudioProcessorManager(unet)
    mgr.setup_processors(verbose=False)
    for p in mgr.level_processors().values():
        p.to(dev)
    B = a.batch
    g = torch.Generator(device="cpu").manual_seed(0)
    ehs = torch.randn(2 * B, 77, 768, generator=g).to(dev, torch.float16)
    audio = {lv: torch.randn(2 * B, 10, 768, generator=g).to(dev, torch.float16) for lv in ("early", "mid", "late")}
    sch = DDIMScheduler()
    sch.set_timesteps(50)
    den = GraphDenoiser(unet, sch, B, a.res, a.res, 7.5, ehs, mgr.get_audio_kwargs(audio))
    with torch.no_grad():
        den.run(torch.randn(B, 4, a.res, a.res, generator=g).to(dev))   # packs weights, captures the step graph
    torch.cuda.synchronize()
    rows, fams, meta = step_ledger(den, a.reps, situ=True)
    txt = format_ledger(rows, fams, meta)
    print(txt, flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(txt)


if __name__ == "__main__":
    main()
