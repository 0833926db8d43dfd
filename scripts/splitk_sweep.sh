# tile-config sweep for the one-tile-per-CU shapes (M=8192, N=512, long K)
set -e
for kind in fwd dgrad; do for K in 2048 1536 512; do for cfg in 4 5 6 9 10 12 13 14; do
timeout -k 5 60 python3 scripts/gemm_one.py --kind $kind --M 8192 --N 512 --K $K --cfg $cfg --splits 1 --reps 30 2>/dev/null | tail -1
done; done; done
