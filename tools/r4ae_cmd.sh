# round-4 check after the BDQN work (via gpurun): the GPU suite, smoke, the default bench line, the other
# configs' lines, the cfg3 profile (kernel trace + env PMC traffic), the cfg5 frame breakdown
set -o pipefail
O=gpurun_out/r4ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/gputest.log 2>&1; echo "pytest rc=$?" >> $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.err || exit 1
done
bash profiles/run_profile.sh r4ae > $O/profile.log 2>&1 || exit 1
bash tools/trace_cfg5.sh r4ae > $O/trace5.log 2>&1 || exit 1
echo done > $O/done
