for e in "X=1" "NLP_GR_WARM=0" "NLP_ETAB=0" ; do echo "=== $e"; env $e STAGES=5 bash tools/gpu_stamps.sh | tail -9 || exit 1; done
