"""bench.py's --graph auto fallback, exercised: the graph capture is made to
raise (as a HIP runtime refusing the capture would), and the bench must run
its eager steps and say so in the line (graph.fallback).

usage: python tools/graph_fallback_check.py   (GPU; a short C2 run)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    gs = sys.modules[pkg.GraphedStep.__module__]

    def refuse(self):
        raise RuntimeError("hipStreamBeginCapture failed (forced by tools/graph_fallback_check.py)")

    gs.GraphedStep._capture = refuse
    sys.argv = ["bench.py", "--config", "C2", "--steps", "20", "--warmup", "3", "--spinup-steps", "20",
                "--diag-steps", "1", "--no-cpu-baseline"]
    out = os.path.join(ROOT, "gpurun_out", "graph_fallback_line.json")
    import contextlib
    import io
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main()
    line = json.loads(buf.getvalue().strip().splitlines()[-1])
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(line, f)
    g = line["graph"]
    assert g["replayed"] is False and "forced" in g.get("fallback", ""), g
    print("fallback ok:", line["value"], line["unit"], "ms", line["ms_per_step"], g)


if __name__ == "__main__":
    main()
