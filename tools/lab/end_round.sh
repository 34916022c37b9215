#!/bin/bash
# end of round: profiles (tools/prof_round.sh: kernel trace + FETCH/WRITE PMC passes of the bench's
# timed step, batched/next_rows trace), then the GPU suite and a default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/prof_round.sh gpurun_out/prof_end || exit $?
NO_TESTS= bash tools/gpu_check.sh
