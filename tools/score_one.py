"""Run the c5 roofline kernel -- the last decoder layer's forward GEMM with
the score epilogue (mmad_fc_fwd_score: y stored, sum (y - ref)^2 row partials)
-- repeatedly at B rows, for rocprofv3 PMC passes (bench_score.py's
score_gemm_roofline launches the same call).
Usage: python tools/score_one.py [batch=65536] [iters=20]"""
import sys
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr
from icra2021_multimodal_ad_amd.model_builder import get_model

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = get_model(types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16"))
nat = m._native
nat.sync_shadow(force=True)
L = nat.layers[-1]
Mp = _native.pad(B)
xin = torch.randn((Mp, L["Kp"]), device="cuda").bfloat16()
ref = torch.randn((Mp, L["Np"]), device="cuda").bfloat16()
out = torch.empty((Mp, L["Np"]), device="cuda", dtype=torch.bfloat16)
rowsq = torch.empty((L["Np"] // 128, Mp), device="cuda")
w = nat.shadow[L["w_off"]:]
bb = nat.params[L["b_off"]:]
for _ in range(iters):
    call("mmad_fc_fwd_score", nat.dt, B, L["N"], L["K"], Mp, L["Np"], L["Kp"], ptr(xin), ptr(w), ptr(bb), 0,
         0.2, None, None, ptr(out), ptr(ref), ptr(rowsq), None, 0, stream_ptr())
torch.cuda.synchronize()
print(f"score GEMM {B}x{L['K']} . {L['N']}x{L['K']}^T x{iters} done", flush=True)
