set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_codecs_fast.py tests/test_gpu_codecs.py tests/test_graph_iid.py > gpurun_out/r06e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06e_tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=indep timeout -k 10 300 python -u tools/inproc_ab.py lib_base lib 20 > gpurun_out/r06e_ab_indep.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06e_ab_indep.txt | tail -8; [ $rc -eq 0 ] || exit $rc
NOPMC= bash tools/gpu_codecs_prof.sh r06e || exit 1
