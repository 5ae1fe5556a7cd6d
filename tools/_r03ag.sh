# round 3 (ag): sharded-step fixed cost at the N = 8 slice (one-rank RCCL group) on the final tree
set -o pipefail
O=gpurun_out/r03_ag; mkdir -p $O
timeout -k 10 300 python3 -u tools/shard_probe.py 8 > $O/shard_probe.txt 2>&1; rc=$?; grep -v "amdgpu.ids\|socket.cpp" $O/shard_probe.txt | tail -4; exit $rc
