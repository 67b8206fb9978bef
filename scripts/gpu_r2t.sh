# row-load shapes micro-benchmark (tools/micro/rgb_rows.hip)
set -u
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/rgb_rows tools/micro/rgb_rows.hip 2> /dev/null
timeout -k 10 120 gpurun_out/rgb_rows > gpurun_out/t_rows.log 2>&1; echo rc=$?
