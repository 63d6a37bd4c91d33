O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "fused_env_act or compact_trainer or act_round or cfg2" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_rollout_$i.json 2> $O/err_$i.log || exit 1
  MS_ENV_ROLLOUT=0 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_perround_$i.json 2>> $O/err_$i.log || exit 1
done
echo done >> $O/job.log
