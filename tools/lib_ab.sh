# Same-box A/B of library builds (tools/build_variant.sh) on one command:
#   LIBS="main u1 u4" TAG=x bash tools/lib_ab.sh python -u tools/compact_probe.py --steps 6 --timed 2
# main = the in-tree build; each run's last JSON line goes to $O/<lib>_<i>.json
set -o pipefail
O=gpurun_out/${TAG:-libab}; mkdir -p $O
export PSAMD_AB=1
for R in 1 2; do for V in ${LIBS:-main}; do
  if [ "$V" = main ]; then unset PSENGINE_LIB_AB; else export PSENGINE_LIB_AB=$PWD/go-libp2p-pubsub_amd/lib/libpsengine_$V.so; fi
  timeout -k 10 300 "$@" > $O/${V}_$R.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "$V $R $(tail -c 400 $O/${V}_$R.json | tr -d '\n' | cut -c1-300)"
done; done
