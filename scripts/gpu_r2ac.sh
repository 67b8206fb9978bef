# VALU instruction rates on gfx950 (tools/micro/valu_rates.hip)
set -u
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/valu_rates tools/micro/valu_rates.hip 2> /dev/null
timeout -k 10 120 gpurun_out/valu_rates > gpurun_out/ac_rates.log 2>&1; echo rc=$?
