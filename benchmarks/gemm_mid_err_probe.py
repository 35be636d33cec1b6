"""gemm_mid vs the 128x128 gemm_bt kernel vs the fp32 reference on mid-M shapes: error statistics."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops
from django_assistant_bot_amd.ops import reference as ref
torch.manual_seed(0)
def bf(*s, scale=1.0): return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)
for (M, N, K) in [(354, 1024, 512), (354, 512, 512), (354, 1024, 512), (316, 512, 512), (384, 4096, 4096), (640, 4096, 14336)]:
    A, B = bf(M, K), bf(N, K, scale=0.05)
    Bs = ops.shuffle_weights(B)
    res = bf(M, N)
    exp = ref.gemm_bt(A.cpu(), B.cpu(), None, None).float()
    mid = ops.kernels.gemm_mid(A, Bs).float().cpu()
    # force the 128 kernel: temporarily raise the gemm_mid floor
    m0 = ops.kernels.GEMM_MID_MIN_M; ops.kernels.GEMM_MID_MIN_M = 1 << 30
    bt128 = ops.gemm_bt(A, Bs, shuffled=True).float().cpu()
    ops.kernels.GEMM_MID_MIN_M = m0
    e = lambda x: (float((x - exp).abs().max()), float((x - exp).abs().mean()))
    exp32 = (A.float() @ B.float().t()).cpu()
    print(json.dumps({"shape": [M, N, K], "mid_vs_fp32": e(mid), "bt128_vs_fp32": e(bt128), "mid_vs_bt128_max": float((mid - bt128).abs().max()),
                      "mid_neq_frac": float((mid != bt128).float().mean()), "out_absmax": float(exp.abs().max()),
                      "exp_vs_exp32": float((exp-exp32).abs().max())}))
# epilogues as the model uses them: residual (o / down), SwiGLU over 8-row [gate | up] groups (gate_up)
for (M, N, K) in [(354, 512, 512), (354, 1024, 512), (640, 4096, 4096)]:
    A, B, res = bf(M, K), bf(N, K, scale=0.05), bf(M, N)
    Bs = ops.shuffle_weights(B)
    exp = ref.gemm_bt(A.cpu(), B.cpu(), None, res.cpu()).float()
    mid = ops.kernels.gemm_mid(A, Bs, residual=res).float().cpu()
    m0 = ops.kernels.GEMM_MID_MIN_M
    ops.kernels.GEMM_MID_MIN_M = 1 << 30
    bt128 = ops.gemm_bt(A, Bs, residual=res, shuffled=True).float().cpu()
    ops.kernels.GEMM_MID_MIN_M = m0
    print(json.dumps({"res_shape": [M, N, K], "mid_vs_ref": float((mid - exp).abs().max()),
                      "bt128_vs_ref": float((bt128 - exp).abs().max()), "mid_neq_ref_frac": float((mid != exp).float().mean()),
                      "bt128_neq_ref_frac": float((bt128 != exp).float().mean())}))
    wg, wu = bf(N // 2, K, scale=0.05), bf(N // 2, K, scale=0.05)
    w8 = ops.shuffle_weights(ops.interleave_gate_up(wg, wu, 8))
    exp = ref.silu_mul(ref.gemm_bt(A.cpu(), torch.cat([wg, wu], 0).cpu())).float()
    mid = ops.kernels.gemm_mid(A, w8, epilogue=ops.EPI_SWIGLU8).float().cpu()
    ops.kernels.GEMM_MID_MIN_M = 1 << 30
    bt128 = ops.gemm_bt(A, w8, epilogue=ops.EPI_SWIGLU8, shuffled=True).float().cpu()
    ops.kernels.GEMM_MID_MIN_M = m0
    print(json.dumps({"swiglu8_shape": [M, N, K], "mid_vs_ref": float((mid - exp).abs().max()),
                      "bt128_vs_ref": float((bt128 - exp).abs().max()), "mid_vs_bt128": float((mid - bt128).abs().max()),
                      "mid_neq_bt_frac": float((mid != bt128).float().mean())}))
