# round-6 call n: N = 1 bench with the public row on both data modes (bf16 + random);
# 2/4/8-rank rehearsals (random mode: engine row vs public row)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/$2.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'})"; }
mkdir -p gpurun_out/r6n
bash tools/gpu/check.sh r6n bench > /dev/null && show r6n bench && \
RANKS=2 bash tools/gpu/check.sh r6n_n2 rehearsal > /dev/null && show r6n_n2 rehearsal && \
RANKS=4 bash tools/gpu/check.sh r6n_n4 rehearsal > /dev/null && show r6n_n4 rehearsal && \
RANKS=8 bash tools/gpu/check.sh r6n_n8 rehearsal > /dev/null && show r6n_n8 rehearsal
