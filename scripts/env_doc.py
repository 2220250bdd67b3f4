"""Regenerate the full switch registry at the end of docs/ENV.md (between the markers) from
docker_dist_nn_amd/switches.py, so the document lists every DNN_* variable the code reads.
Usage: python scripts/env_doc.py [--check]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BEGIN = "<!-- registry:begin (scripts/env_doc.py) -->"
END = "<!-- registry:end -->"


def render() -> str:
    from docker_dist_nn_amd.switches import SWITCHES

    rows = ["## Full registry (generated from `switches.py`)", "",
            "| variable | default | effect |", "|---|---|---|"]
    for name in sorted(SWITCHES):
        default, doc = SWITCHES[name]
        rows.append(f"| `{name}` | `{default}` | {doc.replace('|', '/')} |")
    return "\n".join([BEGIN, *rows, END])


def main():
    path = os.path.join(ROOT, "docs", "ENV.md")
    text = open(path).read()
    block = render()
    if BEGIN in text:
        head, rest = text.split(BEGIN, 1)
        new = head + block + rest.split(END, 1)[1]
    else:
        new = text.rstrip("\n") + "\n\n" + block + "\n"
    if "--check" in sys.argv:
        sys.exit(0 if new == text else 1)
    open(path, "w").write(new)


if __name__ == "__main__":
    main()
