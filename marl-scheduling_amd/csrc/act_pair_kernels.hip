// act_pair_kernels.hip — ms_act_round_free's paired acting kernel (k_act_pair, policy_kernels.hip) in a
// translation unit of its own, so that it alone builds with LLVM's ILP-first machine scheduler
// (build.sh): the cfg3 rollout 12.14 -> 11.88 ms, while the other acting kernels (cfg4's k_act /
// k_act_common) lose with it (profiles/r3f2). policy_kernels.hip is built with MS_SPLIT_PAIR and leaves
// launch_act_round to this unit; with MS_ACT_PAIR_TU it compiles only that launcher and its kernel.
#define MS_ACT_PAIR_TU 1
#include "policy_kernels.hip"
