set -u
O=gpurun_out/r06s9; mkdir -p $O
timeout -k 10 400 python -u tools/sweep.py --config reddit-f41 --grid "hyb_fep=0,1;team_order=0,1" --reps 4 --warm-s 0.5 > $O/reddit_fep.log 2>&1 || exit $?
grep -v amdgpu.ids $O/reddit_fep.log | cut -c1-200 | tail -5
timeout -k 10 400 python -u tools/shard_probe.py --config reddit --world 8 --F 48 --reps 5 --grid "hyb_fep=0,team_order=0;hyb_fep=1,team_order=1;hyb_fep=0,team_order=1;hyb_fep=1,team_order=0" > $O/shard8_fep.log 2>&1 || exit $?
grep -v amdgpu.ids $O/shard8_fep.log | grep step | cut -c1-120
