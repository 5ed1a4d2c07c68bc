"""Per-kernel HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs):
FETCH_SIZE KiB x 2 (gfx950's half count of 16-B/lane streaming reads) x 1024, WRITE_SIZE KiB x
1024 (MI355X_MICROARCH.md, HBM section).  Averages over the dispatches of each kernel name.

    python tools/pmc_kernels.py FETCH_DIR WRITE_DIR [name-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for path in f:
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    keys = sys.argv[3:]
    fe, wr = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    print(f"{'kernel':70s} {'disp':>5s} {'read MB':>10s} {'write MB':>10s}")
    for name in sorted(set(fe) | set(wr)):
        if keys and not any(k in name for k in keys):
            continue
        f = fe.get(name, [])
        w = wr.get(name, [])
        rd = sum(f) / len(f) * 2 * 1024 / 1e6 if f else float("nan")
        wt = sum(w) / len(w) * 1024 / 1e6 if w else float("nan")
        print(f"{name[:70]:70s} {len(f):5d} {rd:10.1f} {wt:10.1f}")


if __name__ == "__main__":
    main()
