#!/bin/bash
# rounds 4a + 4b in one call (the pool is congested: fewer, fuller calls)
cd ${GRAFT_REPO_ROOT:-.}
bash tools/jobs/r4a.sh && bash tools/jobs/r4b.sh
