"""Print ms_per_step (and roofline frac) of the last JSON line of a bench log."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d.get("roofline", {}).get("frac"))
