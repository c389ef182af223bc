#!/bin/bash
# end-of-round profiles: headline (kernel trace + FETCH/WRITE PMC passes) and FC-1000 one-pass big-clique kernel
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
bash tools/profile_session.sh s63/head || exit 1
BENCH_ARGS="--config fc1000" bash tools/profile_session.sh s63/fc || exit 1
