"""Extract the three fixed Perlin permutations (permX / permY / permZ, Noise.hs:60-92) from the
reference source into raytrace_amd/data/perlin_perm.json (data tables, 3 x 256 integers).
Run once in the dev container (the GPU box has no /root/reference); the JSON is committed."""
import json
import os
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/Graphics/Ray/Noise.hs"
text = open(src).read()
out = {}
for name in ("permX", "permY", "permZ"):
    m = re.search(name + r" = A\.fromList A\.Seq\s*\[([^\]]*)\]", text)
    vals = [int(v) for v in re.findall(r"\d+", m.group(1))]
    assert len(vals) == 256 and sorted(vals) == list(range(256)), name
    out[name] = vals
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytrace_amd", "data",
                   "perlin_perm.json")
with open(dst, "w") as f:
    json.dump({"source": "Noise.hs:60-92 (permX, permY, permZ)", **out}, f)
print("wrote", dst)
