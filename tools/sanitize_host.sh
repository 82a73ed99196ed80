#!/bin/bash
# Host-side UndefinedBehaviorSanitizer runs (CPU only; GPU sanitizers are not
# available on this pool): (1) the oracle's C restatement built with
# -fsanitize=undefined under tests/test_oracle.py; (2) the product library with
# its host code (argument validation, workspace sizing, dispatch) built with
# -Xarch_host -fsanitize=undefined under the ABI / host tests, which exercise
# every entry point's error paths without launching a kernel.  Any
# "runtime error" line fails the script.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${TMPDIR:-/tmp}/gs_sanitize
mkdir -p "$T"
gcc -O1 -g -fPIC -fopenmp -ffp-contract=off -fno-fast-math -fsanitize=undefined \
  -fno-sanitize=float-divide-by-zero -shared -o "$T/libgs_oracle_ubsan.so" "$R/oracle/gs_oracle.c" -lm || exit 1
cat > "$T/run_oracle.py" <<PY
import sys
sys.path.insert(0, "$R"); sys.path.insert(0, "$R/tests")
from oracle import oracle as O
O._LIB_PATH = "$T/libgs_oracle_ubsan.so"
O.build = lambda: O._LIB_PATH
import pytest
sys.exit(pytest.main(["-q", "$R/tests/test_oracle.py", "-p", "no:cacheprovider"]))
PY
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux
C=$R/mini-3d-gaussian-splatting_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Xarch_host -fsanitize=undefined -Xarch_host -shared-libsan -Wl,-rpath,$RT -I "$R/include" \
  "$C/gsplat_mi355x.hip" "$C/gs_loss.hip" "$C/gs_densify.hip" -o "$T/libgs_ubsan.so" || exit 1
export UBSAN_OPTIONS=print_stacktrace=1
python "$T/run_oracle.py" > "$T/oracle.log" 2>&1; r1=$?
(cd "$R" && GS_LIB_PATH="$T/libgs_ubsan.so" python -m pytest tests/test_abi.py tests/test_host.py -q -p no:cacheprovider) \
  > "$T/host.log" 2>&1; r2=$?
tail -1 "$T/oracle.log"; tail -1 "$T/host.log"
if grep -h "runtime error" "$T/oracle.log" "$T/host.log"; then exit 1; fi
exit $(( r1 | r2 ))
