set -o pipefail
mkdir -p gpurun_out/r06h
for r in 1 2; do for d in 0 1; do
GS_RR_DMA=$d timeout -k 10 300 python bench.py --steps 2 --warmup 2 --vcycles 0 --config5 0 --config2 0 --cpu-sweeps 0 --newton-iters 3 > gpurun_out/r06h/n_${d}_${r}.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open('gpurun_out/r06h/n_${d}_${r}.json')); n=d['newton']; print('GS_RR_DMA=$d', n['ms_per_iteration'], n['ms_first_iteration'], n.get('ms_per_later_iteration'))"
done; done
GS_RR_DMA=2 timeout -k 10 300 python tools/rr_probe.py
