# free cores skip the P store, BDQN tests, cfg5 line + frame breakdown, ownership fraction
set -o pipefail
O=gpurun_out/r4ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bdqn_gpu.py tests/test_capture_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || exit 1
bash tools/trace_cfg5.sh r4ac > $O/trace5.log 2>&1 || exit 1
echo done > $O/done
echo done > $O/done
