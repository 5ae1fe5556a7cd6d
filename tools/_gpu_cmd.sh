set -o pipefail
O=gpurun_out/r1s18; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || { tail -20 $O/bench1.err; exit 1; }
cat $O/bench1.json
SMX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --n-ops 20000000 > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
cat $O/bench2.json
