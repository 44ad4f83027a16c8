# r03 s52: smoke + GPU suite (main, full size) on the final code, then the 8M R-MAT
# shard probes (8 / 4 / 2 ways) after the hub1 non-temporal id loads
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
SESSION=r03s52 bash tools/r03_tests.sh || exit $?
for w in 8 4 2; do timeout -k 10 240 python tools/shard_probe.py --config rmat-8m --world $w --F 1 > gpurun_out/r03s52/shard8m_$w.log 2>&1 || exit $?; done
echo done
