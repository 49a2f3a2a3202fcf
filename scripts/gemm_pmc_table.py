"""Per-shape table from scripts/gpu_gemm_counters.sh output (gpurun_out/gemmpmc): kernel-trace
average duration (rocprofv3 --kernel-trace --stats) and the median PMC counters of the separate
--pmc passes, derived per MI355X_MICROARCH.md (GRBM_GUI_ACTIVE summed over 8 XCDs; MFMA busy in
SIMD-cycles, 16 per 16x16x32; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles;
FETCH_SIZE x2 on gfx950 for wide streaming reads).
python scripts/gemm_pmc_table.py gpurun_out/gemmpmc name [name ...]"""
import csv
import sys
from pathlib import Path

M0, M2 = 65536, 4096
SHAPES = {  # name: (label, GFLOP, algorithmic read MB, algorithmic write MB)
    "geglu0": ("L0 GEGLU 320->2x1280, M=65536", 2 * M0 * 320 * 2560 / 1e9, (M0 * 320 + 2560 * 320) * 2 / 1e6,
               M0 * 1280 * 2 / 1e6),
    "qkv0": ("L0 QKV 320->960, M=65536", 2 * M0 * 320 * 960 / 1e9, (M0 * 320 + 960 * 320) * 2 / 1e6, M0 * 960 * 2 / 1e6),
    "res0": ("L0 1x1 320->320 + residual, M=65536", 2 * M0 * 320 * 320 / 1e9, (2 * M0 * 320 + 320 * 320) * 2 / 1e6,
             M0 * 320 * 2 / 1e6),
    "l2res": ("L2 1x1 1280->1280 + residual, M=4096", 2 * M2 * 1280 * 1280 / 1e9,
              (2 * M2 * 1280 + 1280 * 1280) * 2 / 1e6, M2 * 1280 * 2 / 1e6),
    "conv0p": ("L0 3x3 320->320 + residual over the zero-bordered source (tile 42), N=16 64^2", 2 * M0 * 320 * 2880 / 1e9,
               (16 * 66 * 66 * 320 + M0 * 320 + 320 * 2880) * 2 / 1e6, M0 * 320 * 2 / 1e6),
    "conv0": ("L0 3x3 320->320 + residual, plain source (tile 40), N=16 64^2", 2 * M0 * 320 * 2880 / 1e9,
              (2 * M0 * 320 + 320 * 2880) * 2 / 1e6, M0 * 320 * 2 / 1e6),
}


def main():
    d = Path(sys.argv[1])
    for name in sys.argv[2:]:
        label, gf, rd, wr = SHAPES[name]
        rows = [r for r in csv.DictReader(open(d / f"{name}_kernel_stats.csv")) if "igemm" in r["Name"]]
        k = max(rows, key=lambda r: float(r["TotalDurationNs"]))
        us = float(k["AverageNs"]) / 1e3
        c = {}
        for ln in open(d / f"{name}_counters.txt"):
            p = ln.split()
            if len(p) >= 2:
                c[p[0]] = float(p[1])
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        simd_cyc = 1024 * cyc
        fetch = 2 * c["FETCH_SIZE"] * 1024 / 1e6
        write = c["WRITE_SIZE"] * 1024 / 1e6
        print(f"== {name}: {label}")
        print(f"   kernel {k['Name']}  avg {us:.1f} us over {k['Calls']} calls")
        print(f"   algorithmic: {gf:.1f} GFLOP -> {gf / us * 1e3:.0f} TF/s = {gf / us * 1e3 / 2500:.3f} of the 2.5 PF MFMA peak; "
              f"bytes {rd + wr:.1f} MB -> {(rd + wr) / us:.2f} TB/s")
        print(f"   clock (GRBM_GUI_ACTIVE / 8 / duration)        {cyc / us / 1e3:.2f} GHz")
        print(f"   MFMA busy (MFMA_BUSY / SIMD-cycles)            {c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cyc:.3f}")
        print(f"   VALU issue (4 x ACTIVE_INST_VALU / SIMD-cyc)   {4 * c['SQ_ACTIVE_INST_VALU'] / simd_cyc:.3f}")
        print(f"   waves waiting (WAIT_ANY / WAVE_CYCLES)         {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
        print(f"   LDS bank-conflict cycles / LDS active          {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        print(f"   L2 hit rate                                    {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
        print(f"   HBM read  FETCH_SIZE x2   {fetch:8.1f} MB vs {rd:7.1f} algorithmic ({fetch / rd:.2f}x)")
        print(f"   HBM write WRITE_SIZE      {write:8.1f} MB vs {wr:7.1f} algorithmic ({write / wr:.2f}x)")
        print(f"   VALU instructions per MFMA {c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA']:.2f}")
        print()


if __name__ == "__main__":
    main()
