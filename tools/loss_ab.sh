#!/bin/bash
# Fused-loss A/B on one box: the loss tests, a bitwise comparison of the
# in-tree library against ab/loss_old.so (gradients must not differ), and a
# rocprofv3 kernel trace of tools/loss_bench.py per library (in-tree + args).
# usage: tools/loss_ab.sh [ab/<lib>.so ...]; then tools/trace_by_grid.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/loss
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_loss.py > $O/pytest.log 2>&1 || exit 1
GS_LIB_PATH=$PWD/ab/loss_old.so timeout -k 10 120 python tools/loss_bench.py /tmp/a.npz > $O/a.log 2>&1 || exit 1
timeout -k 10 120 python tools/loss_bench.py /tmp/b.npz > $O/b.log 2>&1 || exit 1
python tools/bitcmp.py cmp /tmp/a.npz /tmp/b.npz > $O/cmp.log || exit 1
for lib in intree "$@"; do
  n=$(basename $lib .so)
  if [ $lib = intree ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/prof_$n -o run --output-format csv -- python tools/loss_bench.py /tmp/x.npz > $O/prof_$n.log 2>&1 || exit 1
  cp $(find /tmp/prof_$n -name "*kernel_trace.csv") $O/trace_$n.csv
done
