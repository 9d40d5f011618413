set -e
mkdir -p gpurun_out/r05at
for T in 1 2 4 8 16; do timeout -k 10 60 build/probes/tunn_threads $T 50 2000 1350 >> gpurun_out/r05at/tt_b50.jsonl; done
for T in 1 2 4 8 16; do GW_PRIVATE_ENGINES=1 timeout -k 10 60 build/probes/tunn_threads $T 50 2000 1350 >> gpurun_out/r05at/tt_b50_private.jsonl; done
for T in 1 4 16; do timeout -k 10 60 build/probes/tunn_threads $T 256 1000 1350 >> gpurun_out/r05at/tt_b256.jsonl; done
