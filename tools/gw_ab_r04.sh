#!/bin/bash
# A/B: round-4 library + gateway vs current, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05g; mkdir -p $OUT
gcc -O2 -pthread -Iinclude build/variants/r04/udp_gateway.c -Lbuild/variants/r04 -lneptun_gpu -Wl,-rpath,$PWD/build/variants/r04 -o /tmp/gw_r04 || exit 1
gcc -O2 -pthread -Iinclude examples/udp_gateway.c -Lneptun_amd -lneptun_gpu -Wl,-rpath,$PWD/neptun_amd -o /tmp/gw_r05 || exit 1
python3 -c "
import sys, random; sys.path.insert(0,'.')
from tests.test_udp_gateway import ipv4, write_input
rng = random.Random(7)
write_input('/tmp/gin.bin', [ipv4(rng, 1350) for _ in range(262144)], 11, 22, rng.randbytes(32), rng.randbytes(32))
" || exit 1
for rep in 1 2; do
for exe in /tmp/gw_r04 /tmp/gw_r05; do
  for p in 1 4 8; do
    timeout -k 10 120 $exe /tmp/gin.bin /tmp/gout.bin 4096 $p | sed "s#^{#{\"exe\": \"$exe\", #" >> $OUT/ab.jsonl || exit 1
  done
done
done
cat $OUT/ab.jsonl | cut -c1-200
