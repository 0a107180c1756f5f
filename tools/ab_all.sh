#!/bin/bash
# tools/ab_both.sh then tools/ab_lb.sh on the same libraries (one box).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_both.sh "$@" || exit $?
bash tools/ab_lb.sh "$@"
