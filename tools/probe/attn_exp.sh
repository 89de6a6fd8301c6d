set -e
mkdir -p gpurun_out/r19
for cfg in "A" "B:SDIAR_ATTN_HPW=1" "C:SDIAR_ATTN_XREMAP=1" "D:SDIAR_ATTN_HPW=1 SDIAR_ATTN_XREMAP=1" "E:SDIAR_ATTN_HPW=2" "F:SDIAR_ATTN_HPW=4"; do
  name=${cfg%%:*}; envs=""; [ "$cfg" != "$name" ] && envs=${cfg#*:}
  env $envs SDIAR_MAX_BATCH=640 SDIAR_PROF_DETAIL=1 timeout -k 10 200 python tools/kernel_table.py 1 10 > gpurun_out/r19/t_$name.txt 2>&1
  echo "$name $envs $(grep attention gpurun_out/r19/t_$name.txt)" >> gpurun_out/r19/summary.txt
done
