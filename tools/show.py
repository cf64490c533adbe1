"""Print one summary line per bench JSON file (last line of each)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d.get("roofline", {})
    print(f"{f.split('/')[-1]:40s} {d['value']:.3e} upd/s  {d['ms_per_step']:.4f} ms/step  sweeps {d['sweeps']}  "
          f"{r.get('kernel')} x{r.get('launches')} avg {r.get('avg_launch_us', 0):.2f} us  frac {r.get('frac', 0):.3f}")
