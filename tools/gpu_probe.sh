set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/lds_probe > gpurun_out/lds_probe.txt 2>&1; echo "rc=$?"; cat gpurun_out/lds_probe.txt
