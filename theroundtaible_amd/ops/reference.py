"""Plain-PyTorch reference semantics of every hand-written kernel (the numerics oracle).

These run on CPU (unit tests, the GPT-2 CPU plumbing config) and are what the HIP
kernels in ``csrc/`` are tested against. Layouts are the engine's:

* ``k_cache``: allocated ``[num_blocks, n_kv_heads, block_size, head_dim]``, but each
  ``[block, head]`` block is CHUNK-MAJOR in memory: ``[head_dim/32][block_size][32]`` (round 6,
  csrc/common.h ``kc_elem``: a decode-attention K load instruction then reads whole 128-B lines).
  Index it through :func:`k_blocks` / :func:`k_rows` / :func:`write_k`, never as ``[blk, h, off, :]``.
* ``v_cache``: ``[num_blocks, n_kv_heads, head_dim, block_size]`` (V stored transposed per
  block, so the P.V MFMA B-operand is a contiguous load; see csrc/attention_decode.hip)
* ``slot = block_id * block_size + offset``
* ``cos_sin``: ``[max_pos, head_dim]`` fp32 = ``[cos(pos*f_i) | sin(pos*f_i)]`` over
  ``i < head_dim/2`` (Llama rotate-half convention).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

MASK64 = (1 << 64) - 1


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    r = (x.float() + residual.float()).to(x.dtype)
    return rms_norm(r, w, eps), r


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def fused_add_layer_norm(x, residual, w, b, eps):
    r = (x.float() + residual.float()).to(x.dtype)
    return layer_norm(r, w, b, eps), r


def rope_inv_freq(head_dim: int, theta: float, scaling: Optional[tuple] = None) -> Tuple[torch.Tensor, float]:
    """RoPE inverse frequencies (fp64) and the cos / sin magnitude, for the checkpoint's
    ``rope_scaling`` (``models/config.py`` ``ModelConfig.rope_scaling``):

    * ``("linear", factor)``: positions / factor;
    * ``("llama3", factor, low_freq_factor, high_freq_factor, original_max_pos)`` (Llama 3.1 / 3.2):
      wavelengths past ``original / low`` divided by ``factor``, shorter than ``original / high``
      kept, the band between interpolated smoothly;
    * ``("yarn", factor, original_max_pos, beta_fast, beta_slow, attention_factor)`` (YaRN,
      Qwen2.5 long context): per-dimension blend of interpolated / extrapolated frequencies over
      the correction range, cos and sin scaled by ``attention_factor`` (the parser's default:
      0.1 ln(factor) + 1).
    The kernels read the resulting table; nothing else changes."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    mag = 1.0
    if not scaling:
        return inv, mag
    kind = scaling[0]
    if kind == "linear":
        return inv / float(scaling[1]), mag
    if kind == "llama3":
        factor, low_ff, high_ff, orig = (float(v) for v in scaling[1:5])
        wavelen = 2 * math.pi / inv
        low_wl, high_wl = orig / low_ff, orig / high_ff
        out = torch.where(wavelen > low_wl, inv / factor, inv)
        smooth = (orig / wavelen - low_ff) / (high_ff - low_ff)
        mid = (wavelen >= high_wl) & (wavelen <= low_wl)
        return torch.where(mid, (1 - smooth) * out / factor + smooth * out, out), mag
    if kind == "yarn":
        factor, orig, beta_fast, beta_slow, att = (float(v) for v in scaling[1:6])

        def corr_dim(rot):
            return (head_dim * math.log(orig / (rot * 2 * math.pi))) / (2 * math.log(theta))
        low = max(math.floor(corr_dim(beta_fast)), 0)
        high = min(math.ceil(corr_dim(beta_slow)), head_dim - 1)
        if low == high:
            high += 0.001
        ramp = ((torch.arange(head_dim // 2, dtype=torch.float64) - low) / (high - low)).clamp(0, 1)
        extra = 1 - ramp                     # 1: keep the original frequency, 0: interpolate
        out = (inv / factor) * (1 - extra) + inv * extra
        return out, att
    raise ValueError(f"unsupported rope_scaling {scaling!r}")


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None,
                 scaling: Optional[tuple] = None) -> torch.Tensor:
    inv, mag = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos() * mag, f.sin() * mag], dim=-1).float().to(device)


def _rotate(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    # x [T, H, D] float; cs [T, D]
    d2 = x.shape[-1] // 2
    cos, sin = cs[:, None, :d2], cs[:, None, d2:]
    x1, x2 = x[..., :d2], x[..., d2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor],
                   k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                   n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    """Split fused qkv, rotate q/k (if cos_sin given), scatter k/v into the paged cache, return q."""
    T = qkv.shape[0]
    q = qkv[:, :n_heads * head_dim].reshape(T, n_heads, head_dim).float()
    k = qkv[:, n_heads * head_dim:(n_heads + n_kv_heads) * head_dim].reshape(T, n_kv_heads, head_dim).float()
    v = qkv[:, (n_heads + n_kv_heads) * head_dim:].reshape(T, n_kv_heads, head_dim)
    if cos_sin is not None:
        cs = cos_sin[positions.long()]
        q = _rotate(q, cs)
        k = _rotate(k, cs)
    bs = k_cache.shape[2]
    slots = slot_mapping.long()
    blk, off = slots // bs, slots % bs
    write_k(k_cache, blk, off, k)
    v_cache[blk, :, :, off] = v.to(v_cache.dtype)
    return q.to(qkv.dtype)


def k_blocks(k_cache: torch.Tensor) -> torch.Tensor:
    """The chunk-major view of a K cache: ``[num_blocks, n_kv_heads, head_dim/32, block_size, 32]``."""
    nb, hkv, bs, d = k_cache.shape
    return k_cache.view(nb, hkv, d // 32, bs, 32)


def k_rows(k_cache: torch.Tensor, blocks: torch.Tensor) -> torch.Tensor:
    """Key rows of ``blocks`` in order: ``[len(blocks) * block_size, n_kv_heads, head_dim]``."""
    kb = k_blocks(k_cache)[blocks]                       # [n, Hkv, D/32, BS, 32]
    n, hkv, c, bs, w = kb.shape
    return kb.permute(0, 3, 1, 2, 4).reshape(n * bs, hkv, c * w)


def write_k(k_cache: torch.Tensor, blk: torch.Tensor, off: torch.Tensor, k: torch.Tensor) -> None:
    """Store key rows ``k`` ``[T, n_kv_heads, head_dim]`` at (block, offset) pairs."""
    T, hkv, d = k.shape
    k_blocks(k_cache)[blk, :, :, off, :] = k.reshape(T, hkv, d // 32, 32).to(k_cache.dtype)


def set_k_row(k_cache: torch.Tensor, blk: int, head: int, off: int, row: torch.Tensor) -> None:
    """Store one key row ``[head_dim]`` of one KV head (tests)."""
    k_blocks(k_cache)[blk, head, :, off, :] = row.reshape(-1, 32).to(k_cache.dtype)


def _gather_kv(k_cache, v_cache, block_table, n):
    bs = k_cache.shape[2]
    nblk = (n + bs - 1) // bs
    blocks = block_table[:nblk].long()
    k = k_rows(k_cache, blocks)[:n]
    v = v_cache[blocks].permute(0, 3, 1, 2).reshape(nblk * bs, v_cache.shape[1], -1)[:n]
    return k.float(), v.float()


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, ctx_lens: torch.Tensor, scale: float) -> torch.Tensor:
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    for b in range(B):
        n = int(ctx_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], n)     # [n, Hkv, D]
        qb = q[b].float().reshape(Hkv, G, D)
        s = torch.einsum("hgd,nhd->hgn", qb, k) * scale
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgn,nhd->hgd", p, v)
        out[b] = o.reshape(Hq, D).to(q.dtype)
    return out


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      block_tables: torch.Tensor, cu_q: torch.Tensor, start_pos: torch.Tensor,
                      scale: float) -> torch.Tensor:
    """Varlen causal attention: sequence s has queries cu_q[s]:cu_q[s+1] at absolute positions
    start_pos[s] + i, attending to cached keys [0, start_pos[s] + i]."""
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    for s in range(cu_q.shape[0] - 1):
        a, b = int(cu_q[s]), int(cu_q[s + 1])
        if b == a:
            continue
        st = int(start_pos[s])
        n = st + (b - a)
        k, v = _gather_kv(k_cache, v_cache, block_tables[s], n)
        qs = q[a:b].float().reshape(b - a, Hkv, G, D)
        sc = torch.einsum("thgd,nhd->thgn", qs, k) * scale
        qpos = torch.arange(st, n)[:, None]
        kpos = torch.arange(n)[None, :]
        mask = (kpos <= qpos)[:, None, None, :]
        sc = sc.masked_fill(~mask, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        o = torch.einsum("thgn,nhd->thgd", p, v)
        out[a:b] = o.reshape(b - a, Hq, D).to(q.dtype)
    return out


def rope_row_perm(n_rows: int, rope_heads: int, head_dim: int) -> torch.Tensor:
    """Source row of every output row in the pair-interleaved q/k order of the ROPE epilogue:
    row h*D + 2i <- h*D + i, row h*D + 2i + 1 <- h*D + i + D/2 (rows past the q/k heads: identity)."""
    idx = torch.arange(n_rows)
    r = rope_heads * head_dim
    if r:
        h, p = idx[:r] // head_dim, idx[:r] % head_dim
        idx[:r] = h * head_dim + p // 2 + (p % 2) * (head_dim // 2)
    return idx


def rope_bias(b: torch.Tensor, rope_heads: int, head_dim: int) -> torch.Tensor:
    """A q/k/v bias (natural order) as the ROPE epilogue adds it: fp32, in the pair-interleaved
    column order of the shuffled weight (:func:`rope_row_perm`)."""
    return b.float()[rope_row_perm(b.numel(), rope_heads, head_dim).to(b.device)].contiguous()


def fold_gamma(W, gamma=None, rope_heads: int = 0, head_dim: int = 0):
    """W * gamma[None, :] rounded to W's dtype (the RMSNorm weight folded into the next linear),
    rows optionally permuted for the ROPE epilogue (``rope_heads`` leading heads)."""
    out = W.clone() if gamma is None else (W.float() * gamma.float()[None, :]).to(W.dtype)
    if rope_heads:
        out = out[rope_row_perm(W.shape[0], rope_heads, head_dim)].contiguous()
    return out


def skinny_gemm(x, Wf, pro=0, epi=0, res=None, eps=1e-5, x2=None, xout=None):
    """Semantics of csrc/gemm_skinny.hip on the (gamma-folded, row-major) weight ``Wf``:
    y = rsqrt(mean(x^2) + eps)[:, None] * (x @ Wf^T) for the NORM prologue; NORM_ADD (pro=2)
    first forms x = bf16(x + x2) and stores it to ``xout``."""
    if pro == 2:
        x = (x.float() + x2.float()).to(x.dtype)
        if xout is not None:
            xout.copy_(x)
    M, K = x.shape
    xf = x.float()
    y = xf @ Wf.float().t()
    if pro in (1, 2):
        y = y * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    if epi == 2:
        n = Wf.shape[0] // 2
        return (torch.nn.functional.silu(y[:, :n]) * y[:, n:]).to(x.dtype)
    if epi == 1:
        res.copy_((y + res.float()).to(res.dtype))
        return None
    if epi == 3:
        return y  # fp32 pre-rope projection (see skinny_gemm_rope)
    return y.to(x.dtype)


def skinny_gemm_rope(x, Wp, pro, positions, cos_sin, k_cache, v_cache, slots, n_heads, n_kv_heads, head_dim,
                     eps=1e-5, x2=None, xout=None, bias=None):
    """ROPE-epilogue semantics: fp32 projection on the pair-permuted weight (+ the fp32 bias in
    the same column order, :func:`rope_bias`), columns restored to natural order, then RoPE +
    paged K/V scatter with no bf16 rounding in between."""
    y = skinny_gemm(x, Wp, pro, 3, None, eps, x2, xout)
    if bias is not None:
        y = y + bias.float()[None, :]
    perm = rope_row_perm(Wp.shape[0], n_heads + n_kv_heads, head_dim)
    qkv = torch.empty_like(y)
    qkv[:, perm] = y
    q = rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slots, n_heads, n_kv_heads, head_dim)
    return q.to(x.dtype)


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    d = x.shape[-1] // 2
    xf = x.float()
    return (torch.nn.functional.silu(xf[..., :d]) * xf[..., d:]).to(x.dtype)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.gelu(x.float(), approximate="tanh").to(x.dtype)


# ---- sampling -----------------------------------------------------------------------------
# Counter-based RNG shared bit-for-bit with csrc/sampling.hip: u = mix(seed, offset, idx).

def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def uniform_tensor(seed: int, offset: int, n: int) -> torch.Tensor:
    """u in (0,1) for token indices 0..n-1 (vectorized with int64 wraparound arithmetic)."""
    key = _mix64((seed & MASK64) ^ _mix64(offset & MASK64))
    idx = torch.arange(n, dtype=torch.int64)
    z = _mix_t(idx + _to_signed(key))
    # top 24 bits -> (0,1)
    hi = (z >> 40) & 0xFFFFFF
    return (hi.double() + 0.5) / float(1 << 24)


def _to_signed(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


def _mix_t(z: torch.Tensor) -> torch.Tensor:
    def mul(a, c):
        return a * _to_signed(c)  # int64 multiply wraps mod 2^64

    def srl(a, s):  # logical right shift on int64
        return (a >> s) & ((1 << (64 - s)) - 1)

    z = z + _to_signed(0x9E3779B97F4A7C15)
    z = mul(z ^ srl(z, 30), 0xBF58476D1CE4E5B9)
    z = mul(z ^ srl(z, 27), 0x94D049BB133111EB)
    return z ^ srl(z, 31)


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
           seeds: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
    """Greedy when temperature <= 0; else Gumbel-max over the top-k ∩ top-p set.

    Row b's noise is a pure function of (seeds[b], offsets[b], token index); the engine
    passes each knight's token position as its offset, so a knight's sample stream is
    independent of batching, graph replay and round mode."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int64)
    for b in range(B):
        l = logits[b].float()
        t = float(temperature[b])
        if t <= 0:
            out[b] = int(torch.argmax(l))
            continue
        z = (l - l.max()) / t
        allowed = torch.ones(V, dtype=torch.bool)
        k = int(top_k[b])
        if 0 < k < V:
            kth = torch.topk(z, k).values[-1]
            allowed &= z >= kth
        p = float(top_p[b])
        if p < 1.0:
            w = torch.where(allowed, torch.exp(z.double()), torch.zeros((), dtype=torch.float64))
            srt, _ = torch.sort(w, descending=True)
            cs = torch.cumsum(srt, 0)
            cut = int(torch.searchsorted(cs, p * cs[-1]).clamp(max=V - 1))
            thr = srt[cut]
            allowed &= w >= thr
        u = uniform_tensor(int(seeds[b]), int(offsets[b]), V)
        g = -torch.log(-torch.log(u))
        score = torch.where(allowed, z.double() + g, torch.full((), float("-inf"), dtype=torch.float64))
        out[b] = int(torch.argmax(score))
    return out


def decode_prep(slots, offsets, res, ids, positions, block_tables, embed, block_size):
    """Semantics of csrc/decode_step.hip::decode_prep (in place). A position past the block
    table (only after a turn's last step; that slot is never written) maps into block 0."""
    pos = positions.long()
    bi = pos // block_size
    inside = bi < block_tables.shape[1]
    blk = block_tables.long().gather(1, torch.where(inside, bi, 0).unsqueeze(1)).squeeze(1)
    blk = torch.where(inside, blk, 0)
    slots[:len(pos)] = blk * block_size + pos % block_size
    offsets[:len(pos)] = pos + 1
    tok = ids.long().clamp(0, embed.shape[0] - 1)
    res.copy_(embed[tok].to(res.dtype))


def decode_advance(out, ids, positions, ctx_lens, step, nxt, prep=None):
    """Semantics of csrc/decode_step.hip::decode_advance (in place); with prep operands
    (slots, offsets, res, block_tables, embed, block_size) it then runs decode_prep."""
    st = int(step.item())
    if st < out.shape[0]:
        out[st] = nxt
    ids.copy_(nxt)
    positions.add_(1)
    ctx_lens.add_(1)
    step.add_(1)
    if prep is not None:
        slots, offsets, res, bt, embed, bs = prep
        decode_prep(slots, offsets, res, ids, positions, bt, embed, bs)


PAGING_GUARD_CODES = {1: "ctx_len outside [1, max_blocks*block_size]", 2: "block-table entry outside the KV pool",
                      4: "K/V write slot does not match block_tables[pos // block_size]",
                      8: "ctx_len != position + 1"}


def paging_guard(block_tables, ctx_lens, positions, slots, err, num_blocks, block_size):
    """Semantics of csrc/decode_step.hip::paging_guard (err[0] |= violation bits, in place)."""
    code = 0
    maxb = block_tables.shape[1]
    for b in range(ctx_lens.numel()):
        ctx = int(ctx_lens[b])
        if ctx < 1 or ctx > maxb * block_size:
            code |= 1
        nt = min((max(ctx, 0) + block_size - 1) // block_size, maxb)
        row = block_tables[b, :nt]
        if nt and (int(row.min()) < 0 or int(row.max()) >= num_blocks):
            code |= 2
        if positions is not None:
            pos = int(positions[b])
            if pos + 1 != ctx:
                code |= 8
            if slots is not None and pos >= 0 and pos // block_size < maxb:
                want = int(block_tables[b, pos // block_size]) * block_size + pos % block_size
                if int(slots[b]) != want:
                    code |= 4
    err[0] = int(err[0]) | code
