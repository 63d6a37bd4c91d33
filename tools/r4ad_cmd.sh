# sanity of the final tree: the BDQN / capture tests, smoke, the default bench line
set -o pipefail
O=gpurun_out/r4ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bdqn_gpu.py tests/test_capture_gpu.py tests/test_kats.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
echo done > $O/done
