"""Host-only kernel dispatch of every conv launch of a per-launch ledger (bench.py --ops-json), as the current
libcai would choose it (cai_conv_kernel_name; no GPU needed): compares the ledger's kernel with today's choice.
usage: python tools/dispatch_table.py OPS.json [--changed]"""
import ctypes
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))
from compressai import _native  # noqa: E402

lib = _native.lib
pat = re.compile(r"(Conv|ConvT) (\d+)->(\d+) k(\d+) s(\d+) (\d+)x(\d+)->(\d+)x(\d+) B=(\d+)")
DIR = {"conv_fwd": 0, "conv_dgrad": 1, "conv_wgrad": 2}
seen = set()
for l in json.load(open(sys.argv[1]))["launches"]:
    if l["kind"] not in DIR:
        continue
    m = pat.match(str(l["shape"]))
    if not m:
        continue
    kind, cin, cout, k, s, ih, iw, oh, ow, b = m.groups()
    key = (l["kind"], l["shape"])
    if key in seen:
        continue
    seen.add(key)
    g = _native.ConvGeom()
    g.batch, g.in_c, g.out_c = int(b), int(cin), int(cout)
    g.in_h, g.in_w, g.out_h, g.out_w = int(ih), int(iw), int(oh), int(ow)
    g.kernel, g.stride = int(k), int(s)
    g.transposed = int(kind == "ConvT")
    if g.transposed:
        g.pad = int(k) // 2
        g.output_padding = int(oh) - ((int(ih) - 1) * int(s) - 2 * g.pad + int(k))
    else:
        g.pad = int(k) // 2 if int(k) > 1 else 0
        g.output_padding = 0
    now = lib.cai_conv_kernel_name(ctypes.byref(g), _native.BF16, DIR[l["kind"]], 0)
    now = now.decode() if now else "?"
    if "--changed" in sys.argv and now.split("<")[0] in l["kernel"] and now in l["kernel"]:
        continue
    print(f"{l['kind']:10s} {l['shape'][:46]:46s} {l['kernel'][:28]:28s} -> {now}")
