# policy_old sync as one multi-tensor copy: trainer tests, then 20-step bench lines
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "trainer or fullsize or union or compact_variants or dropin or capture" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/bench_$i.json 2> $O/bench.err || exit 1
done
