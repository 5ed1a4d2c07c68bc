"""Per-kernel (full template name) summary of rocprofv3 --pmc passes: cycles per dispatch
(GRBM_GUI_ACTIVE / 8 XCDs), MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / cycles), and the
wave-cycle shares (SQ_WAIT_ANY: parked at s_waitcnt / barrier; SQ_WAIT_INST_ANY: issue stalls;
SQ_ACTIVE_INST_ANY) -- plus instruction counts from a second pass when given.

    python tools/sq_summary.py PASS1_DIR [PASS2_DIR] [--min-cycles 50000]"""
import argparse
import collections
import csv
import glob
import re


def load(d):
    agg = collections.defaultdict(lambda: [0.0, 0])
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k, c = r["Kernel_Name"], r["Counter_Name"]
            agg[(k, c)][0] += float(r["Counter_Value"] or 0)
            agg[(k, c)][1] += 1
    return agg


def name(k):
    m = re.search(r"(gemm_\w+?_kernel)I((?:L[^E]*E)+)E", k)
    if m:
        return m.group(1) + "<" + ",".join(re.findall(r"L[ib](\d+)E", m.group(2))) + ">"
    m = re.search(r"hcr(?:\d+)?(\w+?kernel)", k)
    return m.group(1) if m else k[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--min-cycles", type=float, default=5e4)
    a = ap.parse_args()
    p1 = load(a.dirs[0])
    p2 = load(a.dirs[1]) if len(a.dirs) > 1 else {}
    for k in sorted({k for k, _ in p1}):
        g = lambda d, c: d[(k, c)][0] / max(d[(k, c)][1], 1) if (k, c) in d else float("nan")
        cyc = g(p1, "GRBM_GUI_ACTIVE") / 8
        if not cyc >= a.min_cycles:
            continue
        wave = g(p1, "SQ_WAVE_CYCLES")
        line = (f"{name(k)[:64]:64s} cycles/dispatch {cyc:9.0f}  mfma_busy {g(p1, 'SQ_VALU_MFMA_BUSY_CYCLES') / 1024 / cyc:.3f}"
                f"  wait_any {g(p1, 'SQ_WAIT_ANY') / wave:.3f}  wait_inst {g(p1, 'SQ_WAIT_INST_ANY') / wave:.3f}"
                f"  active {g(p1, 'SQ_ACTIVE_INST_ANY') / wave:.3f}  wait_inst_lds {g(p1, 'SQ_WAIT_INST_LDS') / wave:.3f}")
        if p2:
            line += (f"  | insts lds {g(p2, 'SQ_INSTS_LDS'):.3g} mfma {g(p2, 'SQ_INSTS_MFMA'):.3g}"
                     f" valu {g(p2, 'SQ_INSTS_VALU'):.3g}")
        print(line)


if __name__ == "__main__":
    main()
