# cfg5 frame breakdown (kernel trace), PMC of the cfg3 env / act kernels and of cfg4's gradient kernels
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
bash tools/trace_cfg5.sh r4e > $O/trace5.log 2>&1 || exit 1
bash profiles/run_pmc.sh r4e_cfg3 cfg3 "k_env_step|k_act_pair" > $O/pmc_cfg3.log 2>&1 || exit 1
bash profiles/run_pmc.sh r4e_cfg4 cfg4 "k_ppo_grad|k_own|k_env_step" > $O/pmc_cfg4.log 2>&1 || exit 1
echo done > $O/done
