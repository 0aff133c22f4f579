"""Per-kernel summary of a bench.py --ops-json ledger (time share, roofline efficiency), and optionally the
top-N launches.  usage: python tools/ops_summary.py OPS.json [N]"""
import json
import sys

d = json.load(open(sys.argv[1]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = sum(k["ms"] for k in d["by_kernel"])
print(f"instrumented {tot:.3f} ms over {len(d['launches'])} launches")
for k in d["by_kernel"]:
    print(f"{k['kernel'][:45]:45s} n={k['launches']:3d} ms={k['ms']:.4f} {100 * k['ms'] / tot:5.1f}% "
          f"roof={k['roofline_ms']:.4f} eff={k['roofline_ms'] / max(k['ms'], 1e-9):.2f}")
if top:
    for l in sorted(d["launches"], key=lambda l: -l["ms"])[:top]:
        print(f"  {l['kind'][:10]:10s} {l['kernel'][:32]:32s} {str(l['shape'])[:58]:58s} {l['ms'] * 1e3:7.1f}us "
              f"roof={l['roofline_ms'] * 1e3:6.1f}")
