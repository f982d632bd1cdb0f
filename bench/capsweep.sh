set -o pipefail
for cap in 0 128 256 512; do
  for a in "--steps 20 --warmup 5" "--steps 200 --warmup 40"; do
    echo "cap=$cap $a" >> gpurun_out/cap.log
    XGS_DECODE_PREFILL_CAP=$cap timeout -k 10 240 python bench.py $a 2>/dev/null | grep '^{' >> gpurun_out/cap.log || exit 1
  done
done
