# paired A/B of kernel variants (tools/archive/abtest.sh builds); every variant runs, failures reported
mkdir -p gpurun_out
rc=0
for v in ${AB_VARIANTS:-imm mad lx1 lx2 all1 vf allvf r12 allr}; do
  timeout -k 10 200 tools/abtest_$v ${AB_PAIRS:-80} $v > gpurun_out/ab_$v.log 2>&1 || { echo "AB_FAILED $v (rc $?)"; rc=1; }
  cat gpurun_out/ab_$v.log
done
exit $rc
