# full GPU suite on the act epilogue masks, split hoisting, two-tile compact layer 1, common-row list for compact acting, cfg5 line + frame breakdown, cfg3 line
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bdqn_gpu.py tests/test_capture_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || exit 1
bash tools/trace_cfg5.sh r4o > $O/trace5.log 2>&1 || exit 1


# A/B of MS_UPDATE_STREAMS on one rank, now that the replayed graph records the per-unit-type streams
for i in 1 2; do
  MS_UPDATE_STREAMS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 > $O/us0_$i.json 2> $O/us0_$i.err || exit 1
  MS_UPDATE_STREAMS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 > $O/us1_$i.json 2> $O/us1_$i.err || exit 1
done
echo ab_done > $O/ab_done
timeout -k 10 300 python tools/own_fraction.py > $O/own_fraction.txt 2>&1 || exit 1
echo done > $O/done
