"""Replace one model's rows of docker_dist_nn_amd/parallel/stage_times_gfx950.json with a new
bench/planner_calibrate.py log (JSON lines; other lines ignored).

    python scripts/r6/merge_stage_times.py gpurun_out/cal_mnist-fcnn.log"""
import json
import sys

PATH = "docker_dist_nn_amd/parallel/stage_times_gfx950.json"
new, widths = [], set()
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    new.append([d["widths"], d["a"], d["b"], d["mb"], d["n"], d["ms"]])
    widths.add(tuple(d["widths"]))
doc = json.load(open(PATH))
kept = [r for r in doc["rows"] if tuple(r[0]) not in widths]
doc["rows"] = kept + new
with open(PATH, "w") as f:
    json.dump(doc, f)
print(f"{len(new)} new rows for {sorted(widths)}, {len(kept)} kept")
