SESSION=r02_s10 TEST_GROUPS="tests/test_dist.py tests/test_fullsize.py" bash tools/r02_tests.sh && \
mkdir -p gpurun_out/r02_s10 && \
for w in 2 4 8; do for g in 0 1; do timeout -k 10 200 python tools/shard_probe.py --config rmat-8m --world $w --groups $g >> gpurun_out/r02_s10/shard_probe_8m.log 2>&1 || exit $?; done; done && \
timeout -k 10 200 python tools/shard_probe.py --config rmat-8m --world 1 >> gpurun_out/r02_s10/shard_probe_8m.log 2>&1
