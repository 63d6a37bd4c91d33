# cfg4's offers and compact acceptors in one act launch (k_act_pair<2,2,1,4,4>): tests, then A/B (MS_ACT_UNPAIRED=1)
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "act_round or cfg4 or compact_variants" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_pair_$i.json 2> $O/err.log || exit 1
  MS_ACT_UNPAIRED=1 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_two_$i.json 2>> $O/err.log || exit 1
done
