#!/bin/bash
# Same-box A/B of the dot2 transform (new) against the previous library (old).
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
AB_STEPS=10 tools/ab_libs.sh ${AB_LIBS:-old new1 new2 old new1 new2}
