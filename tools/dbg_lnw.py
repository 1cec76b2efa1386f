"""Stage-2 pwconv h1 (wf_ccf_ffn_stage 1) vs a torch fp64 reference at growing row counts;
run once as is (gemm_lnw) and once with WF_GEMM_NO_LNW=1 (gemm_kc)."""
import sys

import torch

sys.path.insert(0, ".")
import waveformer_amd.network_models as NM  # noqa: E402
from waveformer_amd import _lib, ops  # noqa: E402

_lib.load()
torch.manual_seed(0)
C, hid = 96, 384
mlp = NM.CCF_FFN(C, hid, img_size=(8, 8, 8)).cuda().eval()
with torch.no_grad():
    for p in mlp.parameters():
        p.add_(torch.randn_like(p) * 0.1)
norm2 = torch.nn.LayerNorm(C, eps=1e-6).cuda()
with torch.no_grad():
    norm2.weight.add_(torch.randn_like(norm2.weight) * 0.2)
    norm2.bias.add_(torch.randn_like(norm2.bias) * 0.1)
for (B, S) in [(1, 8), (2, 16), (1, 32), (8, 32)]:
    x = torch.randn(B, S, S, S, C, device="cuda")
    junk = torch.full((2 * 1024 ** 3 // 4,), float("nan"), device="cuda")
    del junk
    st = ops.msfuse([], x, 1e-6)[1]
    with torch.no_grad():
        xh = x
        pw = ops.split_weight(mlp.pwconv.weight, (hid, C), 1)
        fc = ops.split_weight(mlp.fc.weight, prec=1)
        out = torch.empty_like(xh)
        wsb = _lib.query("wf_ccf_ffn_workspace_bytes", B, C, hid, S, S, S, 1)
        work = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
        m = mlp
        args = (xh.data_ptr(), st.data_ptr(), norm2.weight.data_ptr(), norm2.bias.data_ptr(), pw.data_ptr(), m.pwconv.bias.data_ptr(),
                m.norm1.weight.data_ptr(), m.norm1.bias.data_ptr(), float(m.norm1.eps),
                m.dwconv.weight.data_ptr(), m.dwconv.bias.data_ptr(), m.norm2.weight.data_ptr(),
                m.norm2.bias.data_ptr(), float(m.norm2.eps), fc.data_ptr(), m.fc.bias.data_ptr(),
                None, out.data_ptr(), work.data_ptr(), B, C, hid, S, S, S, 1, ops._stream())
        _lib.call("wf_ccf_ffn_stage", 1, *args)
        torch.cuda.synchronize()
        M = B * S ** 3
        h1 = work[: M * hid * 4].view(torch.float32).view(M, hid)
        n2 = torch.nn.functional.layer_norm(x.reshape(M, C).double(), [C], norm2.weight.double(), norm2.bias.double(), 1e-6)
        h = n2 @ m.pwconv.weight.reshape(hid, C).double().t() + m.pwconv.bias.double()
        ref = torch.nn.functional.gelu(torch.nn.functional.layer_norm(
            h, [hid], m.norm1.weight.double(), m.norm1.bias.double(), m.norm1.eps))
        err = ((h1.double() - ref).norm(dim=1) / ref.norm(dim=1))
        bad = (err > 1e-4).nonzero().flatten()
        print(f"B={B} S={S} M={M}: rel-L2 {float((h1.double() - ref).norm() / ref.norm()):.3e} "
              f"max row {float(err.max()):.3e} bad rows {bad.numel()} first {bad[:8].tolist()}",
              flush=True)
