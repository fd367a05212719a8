export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "4096 8" "16384 8" "65536 8" "16384 4" "65536 4"; do
  set -- $cfg
  for w in ppi reddit; do
    st=30; [ $w = reddit ] && st=4
    GAT_BWD_WAVES=$1 GAT_BWD_U=$2 timeout -k 10 200 python tools/train_probe.py $w $st > gpurun_out/ab_${w}_$1_$2.json 2>&1 || exit 1
  done
done
GAT_BWD_KERNEL=stored timeout -k 10 200 python tools/train_probe.py ppi 30 > gpurun_out/ab_ppi_stored.json 2>&1 || exit 1
GAT_BWD_KERNEL=stored timeout -k 10 200 python tools/train_probe.py reddit 4 > gpurun_out/ab_reddit_stored.json 2>&1 || exit 1
