# time tools/call_prof.py <CALL> per library (default + variants), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for lib in binquant_amd/lib/libbinquant_amd.so "$@"; do
    BQ_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/call_prof.py $CALL ${S:-12500} ${T:-2000} | sed "s#^#$lib #" || exit 1
  done
done
