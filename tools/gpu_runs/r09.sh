# uniform vs flow timings, then one rocprofv3 --pmc pass per LDS counter
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/dist
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/dist_probe.py > $OUT/times.log 2>&1; rc=$?
cat $OUT/times.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
for c in SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $R/tools/dist_probe.py > $OUT/$c.log 2>&1; rc=$?
  echo "$c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
