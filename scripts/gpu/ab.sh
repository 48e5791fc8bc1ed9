#!/bin/bash
# GPU box: interleaved same-box A/B of bench.py configurations (fp32 headline,
# secondaries off).  usage: scripts/gpu/ab.sh <reps> "<tag>=<env/args>" ...
# each config is "TAG=ENV1=v ENV2=v -- extra bench args"; prints tag + ms/step per run
reps=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do
  for cfg in "$@"; do
    tag=${cfg%%=*}; rest=${cfg#*=}
    envs=${rest%%--*}; args=""
    [[ "$rest" == *--* ]] && args=${rest#*--}
    env $envs timeout -k 10 200 python -u bench.py --secondary-dtype none --secondary-dcn off $args \
      > "gpurun_out/ab_${tag}_$r.log" 2>&1
    rc=$?
    ms=$(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_${tag}_$r.log" | grep -o '[0-9.]*$')
    echo "$tag rep$r rc=$rc ms_per_step=$ms" | tee -a gpurun_out/ab_summary.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
