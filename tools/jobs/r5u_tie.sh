# auctioneer tie-breaks drawn from the window in one pass: env parity tests, then an A/B against the previous library
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "env_gpu or kats or configs_gpu or compact_variants or dropin or fullsize" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
bash tools/gpu_job.sh r5u ab:old_tie:3:--steps,20,--no-step-kernel
