"""Parse a ZS_DEBUG_CHUNKS=2 dump and walk the chain from unit 0; print where it breaks."""
import re, sys
units = []
for line in open(sys.argv[1]):
    m = re.match(r"\s+unit (\d+) ord (\d+) start (\d+) stop (\d+) end (\d+) code (-?\d+) n_out (\d+) ntok (\d+) tcap (\d+) chain (\d+)", line)
    if m:
        units.append(tuple(int(x) for x in m.groups()))
    elif line.startswith("[zs]") or line.startswith("result"):
        print(line.strip())
act = [u for u in units if u[2] != 0xffffffff]
print("active units", len(act))
codes = {}
for u in act:
    codes[u[5] & 0xff] = codes.get(u[5] & 0xff, 0) + 1
print("codes", codes)
by_start = {u[2]: u for u in act}
u = act[0]
n = 0
while True:
    n += 1
    code = u[5] & 0xff
    if code != 6:
        print("chain ends at member", n, "unit", u, "code", code, "msg", u[5] >> 8)
        break
    nxt = by_start.get(u[4])
    if nxt is None:
        later = [v for v in act if v[2] > u[4]][:3]
        print("no successor at member", n, "unit", u, "next starts", later)
        break
    u = nxt
