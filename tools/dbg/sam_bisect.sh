#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for args in "sam 256 0" "rawam 256 0" "rawsam 256 0" "mixed 128 0"; do
  echo "== $args"
  timeout -k 5 120 python3 -u tools/dbg/sam_bisect.py $args 2>&1 | grep -v "^  File\|^Thread\|^$" | tail -6
  echo "rc=${PIPESTATUS[0]}"
done
echo "== traced mixed 256"
OWRX_SEGV_TRACE=1 timeout -k 5 120 python3 -u tools/dbg/sam_bisect.py mixed 256 0 2>&1 | tail -40
echo "rc=${PIPESTATUS[0]}"
