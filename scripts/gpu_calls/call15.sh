set -uo pipefail
O=gpurun_out/c15; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 1000 python3 -u scripts/tune_in_model.py --preset big --steps 12 --rounds 3 --out $O/tuned_big.json > $O/tune_big.log 2>&1 || { tail -20 $O/tune_big.log; exit 1; }
grep -v amdgpu.ids $O/tune_big.log | tail -40
