# Same-process A/Bs: bash tools/ab_round.sh "c3:lib:lib_d1 c4n:lib:lib_e3 ..."  (c4n = C4 timing-only, no check)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in $1; do
  IFS=: read cfg a b <<< "$spec"
  unset AB_CONFIG AB_NOCHECK
  case $cfg in
    c4) export AB_CONFIG=c4 ;;
    c4n) export AB_CONFIG=c4 AB_NOCHECK=1 ;;
    c3n) export AB_NOCHECK=1 ;;
  esac
  timeout -k 10 200 python3 tools/inproc_ab.py $a $b ${AB_ITERS:-40} > gpurun_out/ab_${cfg}_${a}_${b}.log 2>&1 || { tail -5 gpurun_out/ab_${cfg}_${a}_${b}.log; exit 1; }
  echo "== $cfg"; grep -v amdgpu.ids gpurun_out/ab_${cfg}_${a}_${b}.log
done
