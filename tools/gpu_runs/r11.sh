set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for lib in new prev; do
  if [ $lib = prev ]; then export RSS_TOEPLITZ_LIB=$PWD/tools/librss_toeplitz_prev.so; else unset RSS_TOEPLITZ_LIB; fi
  echo "== $lib rep $rep"
  timeout -k 10 300 python tools/dist_probe.py 2>/dev/null || exit $?
  timeout -k 10 200 python tools/keysearch_bench.py 1024 1048576 uniform || exit $?
  timeout -k 10 200 python tools/keysearch_bench.py 1024 1048576 flow || exit $?
done
done
