#!/bin/bash
# concurrent Tunn callers without sockets (tools/tunn_threads.c): round-4 library vs this tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r05i}; mkdir -p $OUT
gcc -O2 -pthread -Iinclude -DTT_ENGINES tools/tunn_threads.c -Lneptun_amd -lneptun_gpu -Wl,-rpath,$PWD/neptun_amd -o /tmp/tt5 || exit 1
gcc -O2 -pthread -Iinclude tools/tunn_threads.c -Lbuild/variants/r04 -lneptun_gpu -Wl,-rpath,$PWD/build/variants/r04 -o /tmp/tt4 || exit 1
for T in 1 4 8; do
  for v in "/tmp/tt4" "/tmp/tt5" "GW_PRIVATE_ENGINES=1 /tmp/tt5" "WG_TUNN_SPIN_US=0 /tmp/tt5"; do
    timeout -k 10 120 env $v $T 4096 48 | sed "s#^{#{\"variant\": \"$v\", #" >> $OUT/tt.jsonl || exit 1
  done
done
cut -c1-300 $OUT/tt.jsonl
