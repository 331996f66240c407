#!/bin/bash
# round 6: stamp-harness binaries (bin_ab/<name>, built in the container) run alternately, 2 rounds;
# ENVS="A=1 B=2" runs each binary once more per round under those settings
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for b in "$@"; do
    echo "== $b round $r"
    timeout -k 10 60 ./bin_ab/$b || { echo "$b rc=$?"; exit 1; }
    if [ -n "${ENVS:-}" ]; then
      echo "== $b round $r ($ENVS)"
      env $ENVS timeout -k 10 60 ./bin_ab/$b || { echo "$b rc=$?"; exit 1; }
    fi
  done
done
