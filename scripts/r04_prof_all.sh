#!/bin/bash
# One GPU call for the round-4 evidence: 2WL vs occurrence-list phase stamps
# (twl_phases.sh), the product build's kernel stats / traffic / SQ / LDS
# counters (r04_prof.sh), the fetch split of configs 3, 6, 2
# (pmc_fetch_split.sh) and config-4 single-catalog counters
# (pmc_c4_single.sh).  Chained: the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
bash scripts/twl_phases.sh && \
bash scripts/r04_prof.sh && \
bash scripts/pmc_fetch_split.sh "3 6 2" && \
bash scripts/pmc_c4_single.sh 4
