"""Print the batch sweeps of bench JSON lines side by side (tools/sweep_table.py FILE...)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{f}: value {d['value']:.0f} ms/step {d['ms_per_step']} kernel {d['roofline']['kernel_ms_avg']} "
          f"frac {d['roofline']['frac']} ({d['roofline']['bound']})")
    for r in d["extra"]["batch_sweep"] or []:
        print("   B=%4d ms=%.4f kern=%.4f hbm_batch=%.3f hbm_kern=%.3f" % (
            r["batch"], r["ms_per_batch"], r["kernel_ms"], r["hbm_frac_batch"], r["hbm_frac_kernel"]))
