#!/bin/bash
# time the batched PBS stage under several environment settings: time_env.sh "VAR=1" "VAR=0" ...
cd "$(dirname "$0")/../.."
for e in "$@"; do
  echo -n "$e: "
  env $e timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -1 || exit 1
done
