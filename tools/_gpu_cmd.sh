set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_compose.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 bash tools/pmc_passes.sh $PWD/$O/pmc > $O/pmc.log 2>&1; rc=$?; tail -8 $O/pmc.log; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/pmc/summary.json')); print(json.dumps(d['calibration_counter_per_byte']))"
