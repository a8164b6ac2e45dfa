"""Summarise the bench lines of an A/B directory (gpurun_out/<name>/<lib>_<round>.json)."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_[0-9].json"))):
    d = json.load(open(f))
    s = d.get("stats", {})
    print(f"{os.path.basename(f):16s} {d['ms_per_step']:9.3f} ms {d['value']:12.1f} {d['unit']}  "
          f"ber {s.get('ber')} fer {s.get('fer')}")
