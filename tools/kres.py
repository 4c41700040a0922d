"""Register / scratch / occupancy per kernel from hipcc -Rpass-analysis=kernel-resource-usage remarks
(stdin). Usage: see tools/kres.sh."""
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "."
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: +(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if not re.search(pat, r["name"]):
        continue
    g = r.get
    print(f"{r['name'][:64]:64s} VGPR {g('VGPRs', '?'):>4} spill {g('VGPRs Spill', '?'):>3} "
          f"SGPRspill {g('SGPRs Spill', '?'):>4} scratch {g('ScratchSize [bytes/lane]', '?'):>4} "
          f"occ {g('Occupancy [waves/SIMD]', '?'):>2} LDS {g('LDS Size [bytes/block]', '?')}")
