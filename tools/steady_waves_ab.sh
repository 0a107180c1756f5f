#!/bin/bash
# A/B of tier R builds on the steady batches 2..4 (tools/steady_ab.py): each
# library named on the command line (default: the in-tree one)
cd "$GRAFT_REPO_ROOT" || exit 1
[ $# -gt 0 ] || set -- antidote_ccrdt_amd/lib/libccrdt.so
for L in "$@"; do
  CCRDT_LIB=$PWD/$L timeout -k 10 200 python3 tools/steady_ab.py || exit $?
done
