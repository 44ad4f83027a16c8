#!/bin/bash
# The GPU suite against the bounds-checked debug variant of the library:
#   make -C efficient-gnn_amd/csrc VARIANT=debug EXTRA_FLAGS=-DWG_DEBUG_BOUNDS   (here, on the CPU)
#   bash tools/debug_suite.sh <out-name> [pytest args]                             (on the GPU box)
# Every kernel checks gathered ids, wave descriptors, LDS indices and halo rows against their plans
# (WG_DCHECK, csrc/internal.h) and traps with a located message on a violation.  The variant is not
# part of the shipped tree: delete wats_hip/libwats_hip_debug.so after the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1
shift
OUT=gpurun_out/$name
mkdir -p "$OUT"
export WATS_HIP_LIB="$PWD/efficient-gnn_amd/wats_hip/libwats_hip_debug.so"
[ -f "$WATS_HIP_LIB" ] || { echo "no debug library at $WATS_HIP_LIB"; exit 1; }
# the library the suite loads is the bounds-checked one (its message tag is in the code objects)
python -c "import sys; sys.path.insert(0, 'efficient-gnn_amd'); from wats_hip import _lib; \
assert b'WG_DEBUG_BOUNDS' in open(_lib.LIB_PATH, 'rb').read(); print('suite library:', _lib.LIB_PATH)" \
  > "$OUT/debug_lib.txt" 2>&1 || { cat "$OUT/debug_lib.txt"; exit 1; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread "$@" \
  > "$OUT/debug_tests.log" 2>&1
rc=$?
tail -5 "$OUT/debug_tests.log"
grep -m5 "WG_DEBUG_BOUNDS" "$OUT/debug_tests.log"
exit $rc
