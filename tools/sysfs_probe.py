"""List the amdgpu hwmon / pp_dpm_sclk sysfs files bench.PowerSampler reads (no GPU init)."""
import glob
import os

for d in sorted(glob.glob("/sys/class/drm/card*/device")):
    print(d, os.path.realpath(d))
    for f in ("pp_dpm_sclk", "power_dpm_force_performance_level"):
        p = os.path.join(d, f)
        if os.path.exists(p):
            try:
                print("  ", f, open(p).read().strip().replace("\n", " | ")[:200])
            except OSError as e:
                print("  ", f, "unreadable", e)
    for hw in sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*"))):
        for f in sorted(os.listdir(hw)):
            p = os.path.join(hw, f)
            if os.path.isfile(p) and any(f.startswith(x) for x in ("power", "freq", "temp1", "name")):
                try:
                    print("   ", hw.split("/")[-1], f, open(p).read().strip()[:80])
                except OSError as e:
                    print("   ", f, "unreadable", e)
