#!/bin/bash
# Round 4, item 1a: does the execution pass's far-copy traffic cost time?
# A/B of HEAD against a build whose far loads read one fixed L2-resident
# line (wrong bytes, timing only) and one without rounds B, kernel stats of
# both, then the L2 / memory-side counters (TCC) of HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -o pipefail
LIBS="${LIBS:-head farfixed nob}" WLS=c3-decompress bash tools/gpurun/abn.sh || exit 1
LIBS="head farfixed" WLS=c3-decompress bash tools/gpurun/kstats.sh || exit 1
WL=c3-decompress bash tools/gpurun/pmc3.sh || exit 1
