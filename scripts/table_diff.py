"""Convert full copies of the tuned GEMM table into override tables (ops/tuning.py): only the
entries that differ from the default table are kept, so an experiment's table reads as what it
changed. Usage: python scripts/table_diff.py FILE.json [...]  (rewrites in place)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = os.path.join(ROOT, "docker_dist_nn_amd", "ops", "tuned_gfx950.json")


def diff(full: dict, base: dict) -> dict:
    out = {k: v for k, v in full.items() if base.get(k) != v}
    out.update({k: None for k in base if k not in full})
    return out


def main(paths):
    base = json.load(open(DEFAULT))["entries"]
    for p in paths:
        if os.path.realpath(p) == os.path.realpath(DEFAULT):
            print(p, "is the default table itself: skipped (it would be emptied)")
            continue
        doc = json.load(open(p))
        if "override" in doc:
            continue
        ov = {"base": "default", "override": diff(doc.get("entries", {}), base),
              "note": doc.get("note", ""), "date": doc.get("date", "")}
        with open(p, "w") as f:
            json.dump(ov, f, indent=1, sort_keys=True)
            f.write("\n")
        print(p, len(ov["override"]), "entries differ")


if __name__ == "__main__":
    main(sys.argv[1:])
