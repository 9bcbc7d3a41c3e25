# One GPU call for a candidate build: the full GPU test suite on the in-tree library, same-box
# A/Bs against a base build (tools/inproc_ab.py), then the judged set (tools/final_round.sh TAG).
# usage: bash tools/gpu_round.sh <tag> "<config>:<libA>:<libB>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "$@"; do
  IFS=: read cfg A B <<< "$spec"
  AB_CONFIG=$cfg timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-30} > gpurun_out/ab_${TAG}_${cfg}_$B.txt 2>&1
  rc=$?; echo "ab $cfg $A vs $B rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_${TAG}_${cfg}_$B.txt; [ $rc -eq 0 ] || exit $rc
done
bash tools/final_round.sh $TAG || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/final_$TAG/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['encode_ms'], d['decode_ms'], d['dense']['gib_s'], d['c4']['per_gpu_gib_s'], d['c4']['encode_ms'], d['c4']['decode_ms'], d['host']['gib_s'])"
