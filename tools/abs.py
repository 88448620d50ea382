"""Summarise A/B bench logs: value, ms/step and knn launch time of each gpurun_out/<glob> line."""
import glob, json, sys
for pat in sys.argv[1:] or ["gpurun_out/ab_*.log"]:
    for f in sorted(glob.glob(pat)):
        try:
            d = json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1])
        except Exception as e:  # noqa: BLE001
            print(f, "unparsed", e)
            continue
        r = d.get("roofline", {})
        print(f"{f:48s} {d['value']:10.2f} {d['unit']:10s} {d['ms_per_step']:9.3f} ms/step  knn {r.get('avg_launch_ms', 0):.4f} ms  frac {r.get('frac', 0):.3f}")
