set -e
o=gpurun_out/eager_probe.jsonl
: > $o
for a in "--graph 0" "--force-dp 1" "--graph 0" "--force-dp 1"; do timeout -k 10 300 python bench.py --steps 50 --warmup 10 $a 2>/dev/null | grep '^{' >> $o; done
timeout -k 10 300 python scripts/host_time_probe.py > gpurun_out/host_probe.txt 2>&1
