"""Pareto front (queries/s vs recall@1000) of a configs[4] sweep (tools/prune_sweep.py
output): the knobs no other knob beats on both axes.  python tools/pareto.py sweep.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rows = d["rows"]
front = []
for r in rows:
    q, rc = r["device_queries_per_s"], r["recall_at_1000"]
    if not any(o["device_queries_per_s"] >= q and o["recall_at_1000"] >= rc and
               (o["device_queries_per_s"] > q or o["recall_at_1000"] > rc) for o in rows):
        front.append({"min_impact": r["min_impact"], "block_max_factor": r["block_max_factor"],
                      "packed": r["packed"], "k_queries_per_s": round(q / 1e3, 1),
                      "recall_at_1000": round(rc, 4)})
front.sort(key=lambda x: -x["recall_at_1000"])
print(json.dumps({"workload": d["workload"], "front": front}, indent=1))
