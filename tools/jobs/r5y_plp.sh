# price log-prob taken from the table values already loaded (no dependent load): act tests, then A/B
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "act or price or compact_variants or fullsize or dropin" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
bash tools/gpu_job.sh r5y ab:pre_plp:3:--steps,20,--no-step-kernel
