"""Debug helper: encode + decode one device-resident batch shape, report errors/mismatches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import dec_descs, enc_descs
from storb_amd.engine import Engine
from oracle import cfec
nch, n, k, m = map(int, sys.argv[1].split(","))
erased = ((k - 1,) + tuple(range(0, k - 1, 2)))[: m - k]
for u in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4").split(","):
    os.environ["SEC_TILE_U"] = u
    e = Engine(0)
    src = torch.randint(0, 256, (nch * n,), dtype=torch.uint8, device="cuda")
    ed, B = enc_descs(nch, n, k, m)
    par = torch.empty(nch * (m - k) * B, dtype=torch.uint8, device="cuda")
    out = torch.zeros_like(src)
    e.encode_batch(ed, src, par)
    ph = par.cpu().numpy(); sh = src.cpu().numpy()
    ok = all(ph[c*(m-k)*B:(c+1)*(m-k)*B].tobytes() == b"".join(cfec.easy_encode(sh[c*n:(c+1)*n].tobytes(), k, m)[k:]) for c in (0, nch-1))
    print("U", u, "encode vs oracle", ok, flush=True)
    dd, sn, offs = dec_descs(nch, n, k, m, B, src.data_ptr(), par.data_ptr(), erased)
    try:
        e.decode_batch(dd, sn, offs, 0, out)
        print("U", u, "decode equal", torch.equal(out, src), flush=True)
    except Exception as ex:
        print("U", u, "decode error", ex, flush=True)
    e.close()
