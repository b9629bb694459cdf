#!/bin/bash
# LN-epilogue GEMM gangs formed inside XCD groups (RS_LNGANG_XCD=1): parity, interleaved A/B, and
# a FETCH_SIZE pass of each arm (beyond-L2 bytes per row of O-proj / BertOutput)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g2; rm -rf $O; mkdir -p $O
RS_LNGANG_XCD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread -k "lnfuse or fp16x3 or dedup or range_guard or c3_shape or c4_shape" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --utts 100 --steps 2 --warmup 1 --cpu-seconds 0 --fp16-steps 0 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['kinds_ms'])"
}
for r in 1 2; do
  run ticket_r$r RS_LNGANG_XCD=0 || exit 1
  run xcd_r$r RS_LNGANG_XCD=1 || exit 1
done
for arm in 0 1; do
  export RS_LNGANG_XCD=$arm
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch$arm -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 > /dev/null 2> $O/fetch$arm.err || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write$arm -o run --output-format csv -- python bench.py --utts 20 --steps 1 --warmup 0 --cpu-seconds 0 --no-profile --fp16-steps 0 > /dev/null 2> $O/write$arm.err || exit 1
  python tools/pmc_summary.py "$(dirname "$(find $O/fetch$arm -name '*counter_collection.csv' | head -1)")" "$(dirname "$(find $O/write$arm -name '*counter_collection.csv' | head -1)")" $O/traffic$arm.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/traffic$arm.json')); print('gangxcd=$arm', {k: round(d[k]['fetch_size_bytes_per_row']) for k in ('oproj','ffn2','ffn1','qkv')})"
done
