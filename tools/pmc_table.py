#!/usr/bin/env python3
"""Per-kernel table from `tools/gpu.sh pmcsets` output (rocprofv3 --pmc CSVs, one per set).

    python tools/pmc_table.py gpurun_out/pmc [kernel-substring ...]

Derived columns (per dispatch, averaged): MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs /
(GRBM_GUI_ACTIVE / 8 XCDs); LDS conflict share = SQ_LDS_BANK_CONFLICT / 256 CUs / cycles;
wave-wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES; HBM read = 2 x FETCH_SIZE (gfx950 counts half
of wide streaming reads, MI355X_MICROARCH.md), write = WRITE_SIZE; L2 hit = TCC_HIT /
(TCC_HIT + TCC_MISS); VALU per MFMA = SQ_INSTS_VALU / (MFMA busy cycles / 16).
"""
import collections
import csv
import glob
import os
import sys


def _short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "set*", "*counter_collection.csv")) + glob.glob(os.path.join(d, "set*.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if want and not any(w in name for w in want):
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | cycles (per XCD) | MFMA util | LDS conflict | wave wait | VALU/MFMA | HBM read GB | HBM write GB | L2 hit |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, c in vals.items():
        m = {k: sum(v) / len(v) for k, v in c.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc < 1e4:
            continue
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
        util = f"{100 * mf / 1024 / cyc:.1f} %" if mf else "-"
        lds = m.get("SQ_LDS_BANK_CONFLICT")
        ldss = f"{100 * lds / 256 / cyc:.2f} %" if lds is not None else "-"
        w = m.get("SQ_WAIT_ANY"), m.get("SQ_WAVE_CYCLES")
        ws = f"{100 * w[0] / w[1]:.0f} %" if all(w) else "-"
        vm = f"{m['SQ_INSTS_VALU'] / (mf / 16):.2f}" if mf and "SQ_INSTS_VALU" in m else "-"
        rd = f"{2 * m['FETCH_SIZE'] / 1e6:.2f}" if "FETCH_SIZE" in m else "-"
        wr = f"{m['WRITE_SIZE'] / 1e6:.2f}" if "WRITE_SIZE" in m else "-"
        h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
        hs = f"{100 * h / (h + mi):.0f} %" if h is not None and mi is not None else "-"
        short = _short(name)
        print(f"| `{short}` | {cyc:.3g} | {util} | {ldss} | {ws} | {vm} | {rd} | {wr} | {hs} |")
    # wave-cycle breakdown (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES,
    # MI355X_MICROARCH.md rocprofv3 PMC slots) and the issue mix, when those counters were taken
    rows = []
    for name, c in vals.items():
        m = {k: sum(v) / len(v) for k, v in c.items()}
        wc = m.get("SQ_WAVE_CYCLES")
        if not wc or m.get("GRBM_GUI_ACTIVE", 0) / 8 < 1e4:
            continue
        f = lambda k: f"{100 * m[k] / wc:.0f} %" if k in m else "-"  # noqa: E731
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
        co = f"{100 * m['SQ_VALU_MFMA_COEXEC_CYCLES'] / mf:.0f} %" if mf and "SQ_VALU_MFMA_COEXEC_CYCLES" in m else "-"
        rows.append(f"| `{_short(name)}` | {f('SQ_WAIT_ANY')} | {f('SQ_WAIT_INST_ANY')} | "
                    f"{f('SQ_WAIT_INST_LDS')} | {f('SQ_ACTIVE_INST_ANY')} | {f('SQ_ACTIVE_INST_VALU')} | "
                    f"{f('SQ_ACTIVE_INST_LDS')} | {f('SQ_ACTIVE_INST_SCA')} | {co} |")
    if rows and any("SQ_WAIT_INST_ANY" in c or "SQ_ACTIVE_INST_VALU" in c for c in vals.values()):
        print()
        print("| kernel | wait (waitcnt/barrier) | issue stall | LDS issue stall | active | active VALU | active LDS | active scalar | MFMA-VALU coexec / MFMA busy |")
        print("|---|---|---|---|---|---|---|---|---|")
        print("\n".join(rows))


if __name__ == "__main__":
    main()
