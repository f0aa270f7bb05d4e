# round-5 call bd: swarm GPU tests at the final staging rule
set -o pipefail
bash tools/gpu/check.sh r5bd swarm > /dev/null && tail -1 gpurun_out/r5bd/swarm.log
