set -o pipefail
mkdir -p gpurun_out/ring
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "fixture or deterministic or c2_full or c3_full or random_scene or kat or long_tile or odd_image" > gpurun_out/ring/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/ring/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh 3 ab/noring.so ab/ring.so
