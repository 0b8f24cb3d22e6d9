#!/bin/bash
# GPU box: same-box A/B of library variants.  Boxes differ by 2-4%, so only same-box numbers separate
# 1% changes: every variant runs every shape, alternating, PASSES times.
#   variants: VARIANTS="name[:lib][:ENV=V,ENV2=V] ..."  (lib: a file under tfhe-aes-2_amd/dbg/ built by
#             build_variants.sh, or empty for the in-tree library); default: every dbg/*.so as is
#   shapes:   the arguments (scripts/ab/time_stage.py: pbs1, pbs1lat, pbs8, pfks1)
#   CLOCK=1 adds the effective clock of each launch shape; TAE_B sets the batch.
# usage: [PASSES=3] [CLOCK=1] [VARIANTS="..."] scripts/ab/ab.sh shape [shape ...]
cd "$(dirname "$0")/../.."
if [ -z "$VARIANTS" ]; then
  for lib in tfhe-aes-2_amd/dbg/*.so; do n=$(basename $lib .so); VARIANTS="$VARIANTS $n:$n.so:"; done
fi
for pass in $(seq 1 ${PASSES:-3}); do
  for v in $VARIANTS; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
    [ "$rest" = "$v" ] && { lib=""; envs=""; }
    [ "$envs" = "$rest" ] && envs=""
    libpath=""; [ -n "$lib" ] && libpath=$PWD/tfhe-aes-2_amd/dbg/$lib
    for shape in "$@"; do
      line=$(env ${envs//,/ } TAE_CLOCK=${CLOCK:-0} ${libpath:+TAE_LIB_PATH=$libpath} \
             timeout -k 10 ${STEP_TIMEOUT:-240} python scripts/ab/time_stage.py $shape 2>&1)
      rc=$?
      [ $rc -eq 0 ] || { echo "step failed rc=$rc ($name $shape)"; echo "$line" | tail -5; exit 1; }
      echo "$name $(echo "$line" | tail -1)"
    done
  done
done
