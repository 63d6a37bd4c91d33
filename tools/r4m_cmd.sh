# PMC of cfg5's acting kernels (the fused act and the compact layer 1)
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
bash profiles/run_pmc.sh r4m_cfg5 cfg5 "k_bdqn_act|k_bdqn_l1_cores" > $O/pmc_cfg5.log 2>&1 || exit 1
echo done > $O/done
