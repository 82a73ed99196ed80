#!/bin/bash
# Round 6: the replayed (graph) step -- its GPU tests, the frame-path parity
# tests, then the C3 and C2 bench lines.  usage: tools/r06_graph.sh <tag>
set -o pipefail
tag=${1:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_graph_step_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "graph or frame_entry or fixture or deterministic or c2" > "$O/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/c3.log" 2>&1 || { echo "bench failed"; tail -30 "$O/c3.log"; exit 1; }
tail -1 "$O/c3.log" | cut -c1-600
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > "$O/c2.log" 2>&1 || { echo "c2 bench failed"; tail -30 "$O/c2.log"; exit 1; }
tail -1 "$O/c2.log" | cut -c1-400
echo done
