"""TEST INFRASTRUCTURE ONLY -- functional CPU restatement of the WaveFormer reference.

Every function cites the reference line it restates (paths relative to the reference repo
root).  Inputs are (state_dict-like mapping, tensors); nothing here is a torch.nn.Module, so
the oracle shares no code with the product's module tree.  Runs in any float dtype (the golden
tests use float32 like the reference; float64 is used to bound rounding).

Third-party arithmetic restated here:
  * ptwt 0.1.9 (requirements.txt:45) wavedec3 / waverec3 with mode='zero' -- as PyWavelets
    computes it (ptwt is tested against pywt); pinned by PyWavelets 1.1.1 golden vectors.
  * MONAI blocks vendored at monai/networks/blocks/{dynunet_block,unetr_block,patchembedding}.py
  * timm DropPath (identity in eval) / torch.nn defaults.
"""
from __future__ import annotations

import math
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Mapping[str, Tensor]

# ----------------------------------------------------------------------------------------
# wavelets (ptwt.wavedec3 / waverec3, mode='zero'); filter banks are pywt's
# ----------------------------------------------------------------------------------------
_S2 = 0.7071067811865476
FILTERS = {
    # name: (dec_lo, dec_hi, rec_lo, rec_hi), pywt.Wavelet(name) values
    "haar": ((_S2, _S2), (-_S2, _S2), (_S2, _S2), (_S2, -_S2)),
    "db1": ((_S2, _S2), (-_S2, _S2), (_S2, _S2), (_S2, -_S2)),
    "db2": ((-0.12940952255126037, 0.2241438680420134, 0.8365163037378079, 0.48296291314453416),
            (-0.48296291314453416, 0.8365163037378079, -0.2241438680420134, -0.12940952255126037),
            (0.48296291314453416, 0.8365163037378079, 0.2241438680420134, -0.12940952255126037),
            (-0.12940952255126037, -0.2241438680420134, 0.8365163037378079, -0.48296291314453416)),
    "db3": ((0.03522629188570953, -0.08544127388202666, -0.13501102001025458,
             0.45987750211849154, 0.8068915093110925, 0.33267055295008263),
            (-0.33267055295008263, 0.8068915093110925, -0.45987750211849154,
             -0.13501102001025458, 0.08544127388202666, 0.03522629188570953),
            (0.33267055295008263, 0.8068915093110925, 0.45987750211849154,
             -0.13501102001025458, -0.08544127388202666, 0.03522629188570953),
            (0.03522629188570953, 0.08544127388202666, -0.13501102001025458,
             -0.45987750211849154, 0.8068915093110925, -0.33267055295008263)),
    "db4": ((-0.010597401785069032, 0.0328830116668852, 0.030841381835560764,
             -0.18703481171909309, -0.027983769416859854, 0.6308807679298589,
             0.7148465705529157, 0.2303778133088965),
            (-0.2303778133088965, 0.7148465705529157, -0.6308807679298589,
             -0.027983769416859854, 0.18703481171909309, 0.030841381835560764,
             -0.0328830116668852, -0.010597401785069032),
            (0.2303778133088965, 0.7148465705529157, 0.6308807679298589,
             -0.027983769416859854, -0.18703481171909309, 0.030841381835560764,
             0.0328830116668852, -0.010597401785069032),
            (-0.010597401785069032, -0.0328830116668852, 0.030841381835560764,
             0.18703481171909309, -0.027983769416859854, -0.6308807679298589,
             0.7148465705529157, -0.2303778133088965)),
}
DETAIL_KEYS = ("aad", "ada", "add", "daa", "dad", "dda", "ddd")


def _analysis_axis(x: Tensor, dim: int, lo, hi) -> Tuple[Tensor, Tensor]:
    """One analysis step along `dim`, zero extension (pywt MODE_ZERO):
    out[n] = sum_j f[L-1-j] * xpad[2n + j], padl = (2L-3)//2, padr = padl + (len odd)."""
    L = len(lo)
    n = x.shape[dim]
    padl = (2 * L - 3) // 2
    padr = padl + (n % 2)
    x = x.movedim(dim, -1)
    xp = F.pad(x, (padl, padr))
    win = xp.unfold(-1, L, 2)  # (..., nout, L)
    flo = torch.tensor(lo[::-1], dtype=x.dtype, device=x.device)
    fhi = torch.tensor(hi[::-1], dtype=x.dtype, device=x.device)
    a = (win * flo).sum(-1).movedim(-1, dim)
    d = (win * fhi).sum(-1).movedim(-1, dim)
    return a, d


def _synthesis_axis(a: Tensor, d: Tensor, dim: int, rlo, rhi) -> Tensor:
    """One synthesis step along `dim`: y[2n + j] += r[j] c[n], then drop (2L-3)//2 samples
    at both ends (length 2N - L + 2, pywt idwt with MODE_ZERO)."""
    L = len(rlo)
    a = a.movedim(dim, -1)
    d = d.movedim(dim, -1)
    N = a.shape[-1]
    y = torch.zeros(a.shape[:-1] + (2 * N + L - 2,), dtype=a.dtype, device=a.device)
    for j in range(L):
        y[..., j:j + 2 * N:2] += rlo[j] * a + rhi[j] * d
    padl = (2 * L - 3) // 2
    y = y[..., padl:y.shape[-1] - padl]
    return y.movedim(-1, dim)


def dwt3_level(x: Tensor, wavelet: str = "db1") -> Tuple[Tensor, Dict[str, Tensor]]:
    """One 3D level over the last three axes; key char i <-> axis (-3,-2,-1)[i]."""
    lo, hi, _, _ = FILTERS[wavelet]
    out: Dict[str, Tensor] = {}
    za, zd = _analysis_axis(x, -3, lo, hi)
    for zn, zt in (("a", za), ("d", zd)):
        ya, yd = _analysis_axis(zt, -2, lo, hi)
        for yn, yt in (("a", ya), ("d", yd)):
            xa, xd = _analysis_axis(yt, -1, lo, hi)
            out[zn + yn + "a"] = xa
            out[zn + yn + "d"] = xd
    ll = out.pop("aaa")
    return ll, {k: out[k] for k in DETAIL_KEYS}


def wavedec3(x: Tensor, wavelet: str = "db1", level: int = 1) -> List:
    """ptwt.wavedec3(x, wavelet, mode='zero', level=level) -> [LL, dict_coarsest, ..., dict_finest]
    (called at network_models/wave_helper.py:350)."""
    dets = []
    ll = x
    for _ in range(level):
        ll, d = dwt3_level(ll, wavelet)
        dets.append(d)
    return [ll] + dets[::-1]


def idwt3_level(ll: Tensor, det: Dict[str, Tensor], wavelet: str = "db1") -> Tensor:
    _, _, rlo, rhi = FILTERS[wavelet]
    shp = det["aad"].shape
    # pywt waverecn: an LL one sample longer than the details is cropped to them
    ll = ll[tuple(slice(0, s) for s in shp)]
    c = dict(det)
    c["aaa"] = ll
    # undo x (last axis) first, then y, then z
    yz = {}
    for zn in "ad":
        for yn in "ad":
            yz[zn + yn] = _synthesis_axis(c[zn + yn + "a"], c[zn + yn + "d"], -1, rlo, rhi)
    z = {}
    for zn in "ad":
        z[zn] = _synthesis_axis(yz[zn + "a"], yz[zn + "d"], -2, rlo, rhi)
    return _synthesis_axis(z["a"], z["d"], -3, rlo, rhi)


def waverec3(coeffs: Sequence, wavelet: str = "db1") -> Tensor:
    """ptwt.waverec3((LL, dict_coarsest, ..., dict_finest), wavelet)
    (called at network_models/idwt_upsample.py:160)."""
    x = coeffs[0]
    for det in coeffs[1:]:
        x = idwt3_level(x, det, wavelet)
    return x


# ----------------------------------------------------------------------------------------
# attention (network_models/attention.py)
# ----------------------------------------------------------------------------------------
def relative_position_index(ws: int) -> Tensor:
    """attention.py:40-56, including quirk Q2 (depth stride 3*ws-1 instead of (2*ws-1)^2)."""
    r = torch.arange(ws)
    coords = torch.stack(torch.meshgrid([r, r, r], indexing="ij")).flatten(1)  # (3, N)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0) + (ws - 1)
    return rel[..., 0] * (3 * ws - 1) + rel[..., 1] * (2 * ws - 1) + rel[..., 2]


def attention(sd: SD, p: str, x: Tensor, heads: int, ws: int, qk_scale=None) -> Tensor:
    """Attention.forward (attention.py:83-104); x (B_, N, C)."""
    B_, N, C = x.shape
    hd = C // heads
    scale = qk_scale or hd ** -0.5
    qkv = F.linear(x, sd[p + "qkv.weight"], sd.get(p + "qkv.bias"))
    qkv = qkv.reshape(B_, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * scale, qkv[1], qkv[2]
    attn = q @ k.transpose(-2, -1)
    idx = sd[p + "relative_position_index"]
    bias = sd[p + "relative_position_bias_table"][idx.reshape(-1)].reshape(N, N, -1)
    attn = (attn + bias.permute(2, 0, 1).unsqueeze(0)).softmax(-1)
    out = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return F.linear(out, sd[p + "proj.weight"], sd[p + "proj.bias"])


def window_partition(x: Tensor, ws: int) -> Tensor:
    """Block.window_partition (wave_helper.py:450-461)."""
    B, D, H, W, C = x.shape
    x = x.view(B, D // ws, ws, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 5, 2, 4, 6, 7).contiguous().view(-1, ws, ws, ws, C)


# ----------------------------------------------------------------------------------------
# CCF_FFN, PatchMerging (network_models/wave_helper.py)
# ----------------------------------------------------------------------------------------
def ccf_ffn(sd: SD, p: str, x: Tensor) -> Tensor:
    """CCF_FFN.forward (wave_helper.py:260-294); LNs are nn.LayerNorm(c) -> eps 1e-5 (Q5)."""
    B, D, H, W, C = x.shape
    hid = sd[p + "pwconv.weight"].shape[0]
    xp = x.permute(0, 4, 1, 2, 3)
    h = F.conv3d(xp, sd[p + "pwconv.weight"], sd[p + "pwconv.bias"]).reshape(B, hid, -1).transpose(1, 2)
    h = F.gelu(F.layer_norm(h, [hid], sd[p + "norm1.weight"], sd[p + "norm1.bias"], 1e-5))
    h = h.transpose(1, 2).reshape(B, hid, D, H, W)
    h = F.conv3d(h, sd[p + "dwconv.weight"], sd[p + "dwconv.bias"], padding=1, groups=hid)
    h = h.reshape(B, hid, -1).transpose(1, 2)
    h = F.gelu(F.layer_norm(h, [hid], sd[p + "norm2.weight"], sd[p + "norm2.bias"], 1e-5))
    out = F.linear(h, sd[p + "fc.weight"], sd[p + "fc.bias"]).view(B, D, H, W, -1)
    return x + out


def patch_merging(sd: SD, p: str, x: Tensor, eps: float = 1e-6) -> Tensor:
    """PatchMerging.forward (wave_helper.py:173-194) with its duplicated sub-lattices (Q3)."""
    parts = [x[:, 0::2, 0::2, 0::2], x[:, 1::2, 0::2, 0::2], x[:, 0::2, 1::2, 0::2],
             x[:, 0::2, 0::2, 1::2], x[:, 1::2, 0::2, 1::2], x[:, 0::2, 1::2, 0::2],
             x[:, 0::2, 0::2, 1::2], x[:, 1::2, 1::2, 1::2]]
    x = torch.cat(parts, -1)
    x = F.layer_norm(x, [x.shape[-1]], sd[p + "norm.weight"], sd[p + "norm.bias"], eps)
    return F.linear(x, sd[p + "reduction.weight"])


# ----------------------------------------------------------------------------------------
# Block (network_models/wave_helper.py:357-549)
# ----------------------------------------------------------------------------------------
def _dp(t: Tensor, s: Optional[Tensor]) -> Tensor:
    """DropPath with given per-sample factors (timm drop_path: x * mask / keep, the
    `self.drop_path(...)` calls at wave_helper.py:507-508 / :546-547); None = identity."""
    return t if s is None else t * s.view((-1,) + (1,) * (t.dim() - 1))


def block(sd: SD, p: str, x: Tensor, heads: int, level: int, img_size: Sequence[int],
          ms_attention: bool = True, eps: float = 1e-6,
          drop_scales: Optional[Tuple[Tensor, Tensor]] = None):
    """Block.forward -> multi_scale_forward (:470-512) or single_scale_forward (:515-549).
    drop_scales = (attention-branch, FFN-branch) per-sample DropPath factors (training)."""
    s_attn, s_mlp = drop_scales if drop_scales is not None else (None, None)
    D, H, W = img_size
    ws = img_size[0] // (2 ** level)
    B, _, _, _, C = x.shape
    shortcut = x
    x = F.layer_norm(x, [C], sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
    if ms_attention:
        fused = 0
        hfs = []
        for _ in range(max(level, 1)):
            if level > 0:
                ll, det = dwt3_level(x.permute(0, 4, 1, 2, 3).contiguous(), "db1")
                x = ll.permute(0, 2, 3, 4, 1).contiguous()
            osz = x.shape[1:4]
            nW = (osz[0] // ws) * (osz[1] // ws) * (osz[2] // ws)
            win = window_partition(x, ws).view(-1, ws ** 3, C)
            a = attention(sd, p + "attn.", win, heads, ws)
            # quirk Q1: plain reshape back, no inverse permute (wave_helper.py:498-499)
            a = a.view(-1, ws, ws, ws, C).reshape(B, nW, ws, ws, ws, C).reshape(B, *osz, C)
            a = a.permute(0, 4, 1, 2, 3).contiguous()
            if level > 0:
                fused = fused + F.interpolate(a, size=(D, H, W), mode="trilinear")
                hfs.append(det)
            else:
                fused = fused + a
        fused = shortcut + _dp(fused.permute(0, 2, 3, 4, 1), s_attn)
        n2 = F.layer_norm(fused, [C], sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
        out = fused + _dp(ccf_ffn(sd, p + "mlp.", n2), s_mlp)  # Q4: CCF_FFN already adds n2
        if level > 0:
            return out, tuple(reversed(hfs))
        return out
    # single_scale_forward
    x_h = None
    if level > 0:
        c = wavedec3(x.permute(0, 4, 1, 2, 3).contiguous(), "db1", level)
        x, x_h = c[0].permute(0, 2, 3, 4, 1).contiguous(), c[1:]
    osz = x.shape[1:4]
    win = window_partition(x, ws).view(-1, ws ** 3, C)
    a = attention(sd, p + "attn.", win, heads, ws).view(-1, ws, ws, ws, C).reshape(B, *osz, C)
    if level > 0:
        a = F.interpolate(a.permute(0, 4, 1, 2, 3), size=(D, H, W), mode="trilinear")
        a = a.permute(0, 2, 3, 4, 1)
    x = shortcut + _dp(a, s_attn)
    n2 = F.layer_norm(x, [C], sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
    x = x + _dp(ccf_ffn(sd, p + "mlp.", n2), s_mlp)
    if level > 0:
        return x, x_h
    return x


# ----------------------------------------------------------------------------------------
# encoder (network_models/waveformer.py)
# ----------------------------------------------------------------------------------------
def encoder(sd: SD, x: Tensor, *, heads: Sequence[int], depths: Sequence[int],
            levels: Sequence[int] = (3, 2, 1, 0), ms_attention: bool = True,
            prefix: str = "", normalize: bool = True):
    """MultiscaleTransformer.forward_features (waveformer.py:260-322)."""
    p = prefix
    S = x.shape[2]
    # PatchEmbed (monai patchembedding.py:188-214), no norm (patch_norm=False)
    x0 = F.conv3d(x, sd[p + "patch_embed.proj.weight"], sd[p + "patch_embed.proj.bias"], stride=2)
    outs, outs_hf = [], []
    cur = x0.permute(0, 2, 3, 4, 1)
    img = S // 2
    for s in range(4):
        if s > 0:
            cur = patch_merging(sd, f"{p}downsample_{s}.", cur)
            img //= 2
        x_h = None
        for i in range(depths[s]):
            r = block(sd, f"{p}block{s + 1}.{i}.", cur, heads[s], levels[s], (img,) * 3,
                      ms_attention)
            if isinstance(r, tuple):
                cur, x_h = r
            else:
                cur = r
        o = cur.permute(0, 4, 1, 2, 3)
        if normalize:  # proj_out: non-affine layer_norm, eps 1e-5 (waveformer.py:182-204, Q5)
            o = F.layer_norm(o.permute(0, 2, 3, 4, 1), [o.shape[1]]).permute(0, 4, 1, 2, 3)
        outs.append(o)
        if s < 3:
            outs_hf.append(x_h if x_h is not None else ())
    return outs, outs_hf


# ----------------------------------------------------------------------------------------
# decoder blocks (monai/networks/blocks/*, network_models/{idwt_upsample,network_backbone}.py)
# ----------------------------------------------------------------------------------------
def _inorm(x: Tensor) -> Tensor:
    return F.instance_norm(x, eps=1e-5)


def unet_res_block(sd: SD, p: str, x: Tensor) -> Tensor:
    """monai UnetResBlock.forward (dynunet_block.py:98-111), norm 'instance', LeakyReLU(0.01)."""
    out = F.conv3d(x, sd[p + "conv1.conv.weight"], padding=1)
    out = F.leaky_relu(_inorm(out), 0.01)
    out = _inorm(F.conv3d(out, sd[p + "conv2.conv.weight"], padding=1))
    res = x
    if p + "conv3.conv.weight" in sd:
        res = _inorm(F.conv3d(x, sd[p + "conv3.conv.weight"]))
    return F.leaky_relu(out + res, 0.01)


def channel_calibration(sd: SD, p: str, x: Tensor) -> Tensor:
    """ChannelCalibration.forward (network_backbone.py:103-128), InstanceNorm3d (non-affine)."""
    ident = F.conv3d(x, sd[p + "residual.weight"], sd[p + "residual.bias"])
    y = F.relu(_inorm(F.conv3d(x, sd[p + "reduce.weight"], sd[p + "reduce.bias"])))
    y = F.relu(_inorm(F.conv3d(y, sd[p + "conv.weight"], sd[p + "conv.bias"], padding=1)))
    y = _inorm(F.conv3d(y, sd[p + "expand.weight"], sd[p + "expand.bias"]))
    b, c = y.shape[:2]
    se = y.mean(dim=(2, 3, 4))
    se = F.relu(F.linear(se, sd[p + "fc1.weight"], sd[p + "fc1.bias"]))
    se = torch.sigmoid(F.linear(se, sd[p + "fc2.weight"], sd[p + "fc2.bias"])).view(b, c, 1, 1, 1)
    return F.relu(y * se + ident)


def hf_refinement(sd: SD, p: str, x: Tensor) -> Tensor:
    """HFRefinementRes.forward (idwt_upsample.py:39-50), use_sigmoid default True."""
    C = x.shape[1]
    r = F.conv3d(x, sd[p + "conv1.weight"], sd[p + "conv1.bias"], padding=1, groups=C)
    r = F.instance_norm(r, weight=sd[p + "norm.weight"], bias=sd[p + "norm.bias"], eps=1e-5)
    r = F.conv3d(F.relu(r), sd[p + "conv2.weight"], sd[p + "conv2.bias"])
    return x * torch.sigmoid(r)


def idwt_block(sd: SD, p: str, inp: Tensor, skip: Tensor, hf: Sequence[Dict[str, Tensor]],
               hf_refine: bool = False, wavelet: str = "db1") -> Tensor:
    """UnetrIDWTBlock.forward (idwt_upsample.py:138-166)."""
    inp = F.conv3d(inp, sd[p + "conv_lf_block.conv.weight"], padding=1)
    if hf_refine:
        hf = tuple({k: hf_refinement(sd, f"{p}hf_ref.{i}.", d[k]) for k in d}
                   for i, d in enumerate(hf))
    out = waverec3((inp,) + tuple(hf), wavelet)
    out = torch.cat((out, skip), 1)
    return unet_res_block(sd, p + "conv_block.", out)


def projection_upsample(sd: SD, p: str, x: Tensor, stride: int, double_conv: bool) -> Tensor:
    """ProjectionUpsample.forward (wave_helper.py:71-81); GroupNorm(C, C), GELU,
    Upsample(trilinear, align_corners=True)  (Q6)."""
    C = x.shape[1]
    up = F.interpolate(x, scale_factor=stride, mode="trilinear", align_corners=True)
    x1 = F.conv3d(up, sd[p + "conv1.1.weight"], sd[p + "conv1.1.bias"], padding=1, groups=C)
    x1 = F.group_norm(x1, C, sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-5)
    x1 = F.gelu(F.conv3d(x1, sd[p + "conv2.weight"], sd[p + "conv2.bias"]))
    if double_conv:
        x1 = F.gelu(F.conv3d(x1, sd[p + "conv3.0.weight"], sd[p + "conv3.0.bias"]))
        x1 = F.conv3d(x1, sd[p + "conv3.2.weight"], sd[p + "conv3.2.bias"])
    else:
        x1 = F.conv3d(x1, sd[p + "conv3.weight"], sd[p + "conv3.bias"])
    res = F.conv3d(up, sd[p + "res_conv.1.weight"], sd[p + "res_conv.1.bias"])
    return x1 + res


def unetr_up_block(sd: SD, p: str, inp: Tensor, skip: Tensor) -> Tensor:
    """monai UnetrUpBlock.forward (unetr_block.py:83-86): ConvTranspose3d(k2, s2, no bias)."""
    out = F.conv_transpose3d(inp, sd[p + "transp_conv.conv.weight"], stride=2)
    out = torch.cat((out, skip), 1)
    return unet_res_block(sd, p + "conv_block.", out)


def waveformer(sd: SD, x: Tensor, *, heads: Sequence[int], depths: Sequence[int],
               levels: Sequence[int] = (3, 2, 1, 0), hf_refine: bool = False,
               ms_attention: bool = True) -> Tensor:
    """Waveformer.forward (network_backbone.py:380-407)."""
    outs, outs_hf = encoder(sd, x, heads=heads, depths=depths, levels=levels,
                            ms_attention=ms_attention, prefix="waveformer_encoder.")
    enc0 = unet_res_block(sd, "encoder1.layer.", x)
    enc1 = unet_res_block(sd, "encoder2.layer.", outs[0])
    enc2 = unet_res_block(sd, "encoder3.layer.", outs[1])
    enc3 = unet_res_block(sd, "encoder4.layer.", outs[2])
    dec5 = channel_calibration(sd, "encoder10.", outs[3])
    dec4 = idwt_block(sd, "decoder4.", dec5, enc3, outs_hf[-1], hf_refine)
    dec3 = idwt_block(sd, "decoder3.", dec5, enc2, outs_hf[-2], hf_refine)
    dec2 = idwt_block(sd, "decoder2.", dec5, enc1, outs_hf[-3], hf_refine)
    up4 = projection_upsample(sd, "learnable_up4.", dec4, 4, True)
    up3 = projection_upsample(sd, "learnable_up3.", dec3, 2, False)
    dec1 = unetr_up_block(sd, "decoder1.", torch.cat([up4, up3, dec2], 1), enc0)
    return F.conv3d(dec1, sd["out.conv.conv.weight"], sd["out.conv.conv.bias"])
