set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/pstream benchmarks/persistent_stream_probe.hip
timeout -k 10 120 /tmp/pstream > gpurun_out/r2_pstream.log 2>&1 || { echo PROBE_FAIL; cat gpurun_out/r2_pstream.log; exit 1; }
cat gpurun_out/r2_pstream.log
