#!/bin/bash
# Round 6, session G (round-end evidence, part 1): the whole GPU suite, smoke, the default
# bench line.  Part 2 (tools/gpu_r06h.sh): rocprofv3 summaries and PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STAGES="tests smoke bench" TAILN=12 bash tools/gpu_session.sh
