#!/bin/bash
# GPU-box routine for a round's closing artefacts: full parity suite, smoke(), the default bench line (with
# CPU baseline and its per-launch table), a rocprofv3 kernel-stats pass, the two PMC traffic passes of the bench
# line's roofline launch (pinned by kind:index, so both passes count the same launch), and the other configs.
# usage (via gpurun): bash tools/final_check.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/fin_${tag}_test.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/fin_${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --ops-json $out/fin_${tag}_ops.json > $out/fin_${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/fin_${tag}_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $out/fin_${tag}_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
rep=$(python3 - "$out/fin_${tag}_bench.log" "$out/fin_${tag}_ops.json" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
kind, shape = json.loads(line)["roofline"]["launch"].split(": ", 1)
rows = json.load(open(sys.argv[2]))["launches"]
same = [r for r in rows if r["kind"] == kind]
print(f"{kind}:{[r['shape'] for r in same].index(shape)}")
EOF
) || exit 1
echo "$rep" > $out/fin_${tag}_replay.txt
bash tools/pmc_traffic.sh $rep || exit 1
# the big stride-2 convs' counter records: g_a[2] fwd (conv_halo_kernel<5>, 1024 blocks),
# g_s[4] fwd and g_a[2] dgrad (conv_halo_quad_kernel)
bash tools/pmc_traffic.sh conv_fwd:1 conv_fwd:12 conv_dgrad:12 || exit 1
bash tools/bench_models.sh fin_$tag
