"""Derived per-launch metrics from scripts/gpu_counters.sh summaries (median counters).
python scripts/pmc_derive.py <name>_counters.txt <avg_us> [n_simd]
Units (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE summed over the 8 XCDs (cycles = /8);
SQ_VALU_MFMA_BUSY_CYCLES in SIMD-cycles (16 per 16x16x32 MFMA) summed over SIMDs;
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles summed over waves."""
import sys

c = {}
for ln in open(sys.argv[1]):
    p = ln.split()
    if len(p) >= 2 and p[0].isupper() or (p and p[0].startswith(("SQ_", "TCC_", "GRBM_"))):
        c[p[0]] = float(p[1])
us = float(sys.argv[2])
nsimd = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
cyc = c["GRBM_GUI_ACTIVE"] / 8
print(f"kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs)   {cyc:12.0f}  -> clock {cyc / us / 1e3:.2f} GHz at {us:.1f} us")
print(f"MFMA busy  (SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles)  {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (nsimd * cyc):6.3f}")
print(f"VALU issue (4 x SQ_ACTIVE_INST_VALU / SIMD-cycles)   {4 * c['SQ_ACTIVE_INST_VALU'] / (nsimd * cyc):6.3f}")
print(f"waves waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)        {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:6.3f}")
print(f"LDS bank-conflict cycles / LDS active cycles        {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:6.3f}")
print(f"L2 hit rate (TCC_HIT / (HIT + MISS))                {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):6.3f}")
print(f"MFMA instructions per launch                        {c['SQ_INSTS_MFMA']:12.0f}")
