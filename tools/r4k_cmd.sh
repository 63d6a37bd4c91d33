# full GPU suite on the precomputed W1_c F in the compact layer 1, cfg5 line + frame breakdown, cfg3 line
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bdqn_gpu.py tests/test_capture_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || exit 1
bash tools/trace_cfg5.sh r4k > $O/trace5.log 2>&1 || exit 1

echo done > $O/done
