"""Debug: one build variant against the default build on C2, fresh buffers each (not product)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import dec_descs, enc_descs  # noqa: E402
from storb_amd.engine import Engine  # noqa: E402

tag, u = sys.argv[1], sys.argv[2]
nch, n, k, m = int(sys.argv[3]) if len(sys.argv) > 3 else 64, 1 << 20, 4, 6
src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
ed, B = enc_descs(nch, n, k, m)
res = {}
for name, lib in (("default", None), (tag, f"storb_amd/lib/libstorbec_{tag}.so")):
    os.environ["SEC_TILE_U"] = u
    e = Engine(0, lib_path=lib)
    par = torch.zeros(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
    out = torch.zeros_like(src)
    dd, sn, offs = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), (1, 3))
    for rep in range(3):
        par.zero_()
        out.zero_()
        e.encode_batch(ed, src, par)
        e.decode_batch(dd, sn, offs, 0, out)
        res.setdefault(name, []).append((par.clone(), bool(torch.equal(out, src))))
for name, runs in res.items():
    print(name, "decode ok per rep:", [ok for _, ok in runs],
          "parity == default rep0:", [bool(torch.equal(p, res["default"][0][0])) for p, _ in runs],
          "nonzero parity bytes:", [int((p != 0).sum()) for p, _ in runs])
