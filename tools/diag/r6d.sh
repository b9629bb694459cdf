#!/bin/bash
# Round 6: multi-rank rehearsal of the bench on ONE GPU (2 ranks sharing GPU 0, gloo exchange):
# bench.py --gpus 2 through its own launcher, then the driver's torch.distributed.run form.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6d; rm -rf $O; mkdir -p $O
A="--utts 40 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 --finetune-steps 20"
RS_BENCH_DEVICE=0 RS_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 $A > $O/launcher.json 2> $O/launcher.err && \
RS_BENCH_DEVICE=0 RS_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $A > $O/torchrun.json 2> $O/torchrun.err
rc=$?
for f in launcher torchrun; do echo "== $f: $(wc -l < $O/$f.json) line(s)"; python -c "
import json,sys
for l in open('$O/$f.json'):
    l=l.strip()
    if l.startswith('{'):
        r=json.loads(l); print(r['n_gpus'], r['value'], r['ms_per_step'], r['config']['parallelism'], r['config']['forwards_per_step'], r['config']['forwards_rank0_step'], r['rerank'])
"; done
tail -n 5 $O/launcher.err $O/torchrun.err
exit $rc
