set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04e STEPS=sweep SWEEP_ARGS="--config C4-sk-2005 --metrics JAC --hubs 16 --cpu-hubs= --reps 2 --envs NLP_HB_XP=0;NLP_HB_XP=1;NLP_HB_XP=2;NLP_HB_XP=4;NLP_HB_XP=7" tools/gpu_r04.sh || exit 1
TAG=r04e SPEC=C4-sk-2005:JAC:16 timeout -k 10 900 tools/gpu_pmc_call.sh
