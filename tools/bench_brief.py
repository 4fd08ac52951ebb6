"""One-line summary of bench.py JSON logs: value, ms/step and per-stage ms per launch.
    python tools/bench_brief.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    st = d.get("stages_ms_per_launch", {})
    m = d.get("stage_rooflines", {}).get("match", {})
    print(f"{f}: {d['value']:.0f} fps {d['ms_per_step']:.3f} ms | " + " ".join(f"{k} {v:.3f}" for k, v in st.items())
          + (f" | match frac {m.get('frac')}" if m else ""))
