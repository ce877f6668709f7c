import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
print({k: v for k, v in os.environ.items() if "VISIBLE" in k or "HIP" in k or "HSA" in k or "ROC" in k})
mode = sys.argv[1]
from storb_amd.engine import Engine, get_engine
if mode == "engine_first":
    e = Engine(0)
    print("engine ok")
elif mode == "host_call_first":
    e = get_engine()
    print(e.encode_host([b"x" * 100000], [(4, 6)])[0][0][:4])
import torch
print("torch devices", torch.cuda.device_count(), torch.cuda.is_available())
x = torch.zeros(4, device="cuda")
print("torch ok", x.sum().item())
