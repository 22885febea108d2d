"""Op dispatch: hand-written HIP/CDNA4 kernels on GPU tensors, PyTorch reference on CPU.

GPU tensors ALWAYS go to the native extension ``theroundtaible_amd._C`` (built
in-tree by ``csrc/build.py``); if it is missing on a GPU box the op raises instead
of silently falling back, so a test can never pass on eager PyTorch while claiming
to exercise the kernels. (``ROUNDTABLE_ALLOW_TORCH_FALLBACK=1`` exists only for
debugging a broken build.)
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import reference as ref

_NATIVE = None
_NATIVE_ERR: Optional[BaseException] = None


def native():
    """The compiled extension module (raises if it cannot be imported)."""
    global _NATIVE, _NATIVE_ERR
    if _NATIVE is None and _NATIVE_ERR is None:
        try:
            from .. import _C  # type: ignore
            _NATIVE = _C
        except BaseException as e:  # noqa: BLE001
            _NATIVE_ERR = e
    if _NATIVE is None:
        raise RuntimeError(f"theroundtaible_amd._C (HIP kernels) is not built/importable: {_NATIVE_ERR}. "
                           f"Run `python csrc/build.py` (or __graft_entry__.build()).")
    return _NATIVE


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def _use_native(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if os.environ.get("ROUNDTABLE_ALLOW_TORCH_FALLBACK") == "1" and not native_available():
        return False
    return True


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    if _use_native(x):
        out = torch.empty_like(x)
        native().rms_norm(out, x, w, eps)
        return out
    return ref.rms_norm(x, w, eps)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (rmsnorm(x + residual), x + residual). On GPU ``residual`` is updated in place."""
    if _use_native(x):
        out = torch.empty_like(x)
        native().fused_add_rms_norm(out, x, residual, w, eps)
        return out, residual
    return ref.fused_add_rms_norm(x, residual, w, eps)


def layer_norm(x, w, b, eps):
    if _use_native(x):
        out = torch.empty_like(x)
        native().layer_norm(out, x, w, b, eps)
        return out
    return ref.layer_norm(x, w, b, eps)


def fused_add_layer_norm(x, residual, w, b, eps):
    if _use_native(x):
        out = torch.empty_like(x)
        native().fused_add_layer_norm(out, x, residual, w, b, eps)
        return out, residual
    return ref.fused_add_layer_norm(x, residual, w, b, eps)


def rope_and_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor],
                   k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                   n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    if _use_native(qkv):
        q = torch.empty(qkv.shape[0], n_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
        native().rope_and_cache(q, qkv, positions, cos_sin if cos_sin is not None else torch.empty(0, device=qkv.device),
                                k_cache, v_cache, slot_mapping, n_heads, n_kv_heads, head_dim)
        return q
    return ref.rope_and_cache(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, n_heads, n_kv_heads, head_dim)


MAX_GROUP_COLS = 16      # MFMA columns a shared-prefix group's query heads may fill (n * G)


# attention plan row: 8 header ints + 512 block ids (the 8 waves x 64 lanes of an item's first
# block-id fetch; an item with more tiles reads the rest from the block tables)
PLAN_STRIDE = 8 + 512


def plan_enabled() -> bool:
    """Per-step attention plan (``ROUNDTABLE_ATTN_PLAN=0`` turns it off: A/B)."""
    return os.environ.get("ROUNDTABLE_ATTN_PLAN", "1") != "0"


class DecodeWorkspace:
    """Split-KV scratch for paged decode (static: allocated once, reused inside hipGraphs).

    ``max_group``: largest shared-prefix group (knights reading the same KV prefix, see
    :func:`decode_groups`); each (sequence, head) then receives up to ``max_group * max_splits``
    partials, so the partial buffers are strided by ``slot_stride`` = that product."""

    def __init__(self, max_batch: int, n_heads: int, head_dim: int, max_splits: int, device, max_group: int = 1):
        self.max_splits = max_splits
        self.max_group = max(1, max_group)
        self.slot_stride = max_splits * self.max_group
        self.partial_o = torch.empty(max_batch * n_heads * self.slot_stride * head_dim, dtype=torch.float32,
                                     device=device)
        self.partial_ml = torch.empty(max_batch * n_heads * self.slot_stride * 4, dtype=torch.float32, device=device)
        # per-(sequence, kv head) split arrival counters; the kernel re-arms them to 0 itself.
        # Sized by n_heads (>= n_kv_heads) so one workspace serves every GQA ratio.
        self.counters = torch.zeros(max_batch * n_heads, dtype=torch.int32, device=device)
        # persistent / experiment kernels: phase counters (self-re-arming) and the poll-expiry flag
        # (tools/experiments: decode_layer.hip, combine_o.hip)
        self.sync = torch.zeros(8, dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        # per-step attention work plan (attn_plan): per item (sequence, split) a header + the
        # item's block ids; written once per decode step, read by every layer's launch
        self.plan_stride = PLAN_STRIDE
        self.plan = torch.empty(max_batch * max_splits * PLAN_STRIDE, dtype=torch.int32, device=device)
        self.planned = False


_CUS: dict = {}


def device_cus(device=None) -> int:
    """Compute units of ``device`` (the current GPU; 256 = MI355X when no GPU is visible)."""
    if not torch.cuda.is_available():
        return 256
    idx = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    if idx not in _CUS:
        _CUS[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count)
    return _CUS[idx]


def decode_splits(batch: int, n_kv_heads: int, num_cus: Optional[int] = None, max_splits: int = 64,
                  grouped: bool = False) -> int:
    """Split-KV count fixed per (batch bucket, kv heads): at most one 8-wave workgroup per CU
    (measured on MI355X, profiles/r01_microbench_v1.log: B=3, ctx 6000 -> 8 splits 22 µs,
    11 splits 27 µs, 16 splits 28 µs; extra workgroups only add hand-off round trips).

    The kernel derives each split's key range from the *runtime* context length, so one
    captured hipGraph serves every length (splits past the end are empty and skipped by the
    combine) — no re-capture as a knight's discussion grows."""
    # grouped (shared-prefix) decode takes the whole chip too. Round 2 measured 3/4 of the CUs best
    # for the 3-knight table (B=3, shared 22K/40K: 8 splits 30.8/42.7 us vs 10 splits 31.7/43.8,
    # r2_gattn_v1.log); with the round-5 copy-free K/V loop the whole chip wins (8 -> 10 splits:
    # 29.0 -> 28.2 / 42.4 -> 40.9 us; driver-config bench 837.1 -> 840.1 tok/s, mean of three
    # same-box passes), and for larger tables by far (16 knights: 1 -> 2 splits 47.5 -> 29.9 us;
    # profiles/r05/attn_splits_large_tables.md).
    # A lone sequence (B = 1: sequential rounds) shares nothing, so it takes the whole chip: B = 1,
    # Llama-3-8B, 10K / 25K / 40K keys: 24 splits 15.9 / 26.3 / 36.8 us, 32 splits 15.0 / 25.9 /
    # 35.7 (profiles/r03/attn_b1_splits.md)
    num_cus = device_cus() if num_cus is None else num_cus
    # ROUNDTABLE_GROUPED_CU_FRACTION: A/B knob for the grouped share of the CUs (default: all)
    frac = float(os.environ.get("ROUNDTABLE_GROUPED_CU_FRACTION", "1.0"))
    cus = int(num_cus * frac) if grouped and batch > 1 else num_cus
    want = cus // max(1, batch * n_kv_heads)        # never more workgroups than CUs: a second
    return int(max(1, min(max_splits, want)))       # wave of workgroups doubles the tail


def decode_groups(group_of: list, shared_blocks: list, G: int) -> Tuple[torch.Tensor, int]:
    """Per-sequence ``[B, 3]`` int32 ``{first sequence, group size n, shared full blocks}`` for
    the shared-prefix decode kernel, from a group label per sequence (members must be
    consecutive; ``None`` = alone) and each group's shared block count. Groups wider than the
    MFMA columns (n * G > 16) are cut into consecutive sub-groups of the same prefix. Returns
    the table and the largest n."""
    B = len(group_of)
    out = torch.zeros(B, 3, dtype=torch.int32)
    cap = max(1, MAX_GROUP_COLS // max(1, G))
    b, nmax = 0, 1
    while b < B:
        e = b + 1
        if group_of[b] is not None:
            while e < B and group_of[e] == group_of[b] and e - b < cap:
                e += 1
        n = e - b
        sh = int(shared_blocks[b]) if n > 1 else 0
        if sh <= 0:
            n, e, sh = 1, b + 1, 0
        for i in range(b, e):
            out[i] = torch.tensor([b, n, sh], dtype=torch.int32)
        nmax = max(nmax, n)
        b = e
    return out, nmax


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, ctx_lens: torch.Tensor, scale: float,
                           num_splits: int = 1, workspace: Optional[DecodeWorkspace] = None,
                           out: Optional[torch.Tensor] = None, groups: Optional[torch.Tensor] = None,
                           planned: bool = False) -> torch.Tensor:
    """``groups`` (optional, device ``[B, 3]`` int32 from :func:`decode_groups`): sequences whose
    block tables share leading blocks decode those keys once for the whole group. The result is
    identical to decoding every sequence alone (the fp32 oracle ignores ``groups``).
    ``planned``: the workspace holds this step's :func:`attn_plan` for exactly these arguments."""
    if _use_native(q):
        if out is None:
            out = torch.empty_like(q)
        G = q.shape[1] // k_cache.shape[1]
        if workspace is None:
            workspace = DecodeWorkspace(q.shape[0], q.shape[1], q.shape[2], max(1, num_splits), q.device,
                                        max_group=MAX_GROUP_COLS // G if groups is not None else 1)
        if groups is not None and (workspace.max_group < MAX_GROUP_COLS // G or workspace.max_splits < num_splits):
            raise ValueError(f"decode workspace too small for shared-prefix groups (max_group "
                             f"{workspace.max_group} < {MAX_GROUP_COLS // G})")
        plan = workspace.plan if planned else None
        native().paged_attention_decode(out, q, k_cache, v_cache, block_tables, ctx_lens, scale,
                                        int(num_splits), workspace.partial_o, workspace.partial_ml,
                                        workspace.counters, groups,
                                        workspace.slot_stride if groups is not None else 0, False,
                                        plan, workspace.plan_stride if planned else 0)
        return out
    return ref.paged_attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)


def attn_plan(block_tables: torch.Tensor, ctx_lens: torch.Tensor, num_splits: int, workspace: DecodeWorkspace,
              n_heads: int, n_kv_heads: int, groups: Optional[torch.Tensor] = None, batch: Optional[int] = None) -> bool:
    """Write the per-step decode-attention work plan into ``workspace`` (csrc/attention_decode.hip
    attn_plan_kernel): every layer's :func:`paged_attention_decode` of this step (same block tables,
    lengths, groups, splits) then passes ``planned=True`` and starts its K/V stream one dependent
    round trip earlier. Returns whether a plan was written (GPU + native + enabled)."""
    if workspace is None or not block_tables.is_cuda or not native_available() or not plan_enabled():
        return False
    B = int(batch if batch is not None else ctx_lens.numel())
    if B * num_splits * workspace.plan_stride > workspace.plan.numel():
        return False
    native().attn_plan(workspace.plan, workspace.plan_stride, block_tables, ctx_lens, groups, B, int(n_heads),
                       int(n_kv_heads), int(num_splits))
    return True


def prefill_tile_map(cu_q: torch.Tensor, rows_per_tile: int, start_pos=None) -> torch.Tensor:
    """[n_tiles, 2] int32 (sequence, first row) work list for the varlen prefill kernel,
    heaviest tiles first: under the causal mask a tile's work grows with its last key, and
    workgroups start in list order, so the long tiles begin at once and the short ones fill
    the tail (T=4096: 1.3x less time than row order)."""
    items = []
    cq = cu_q.tolist()
    sp = start_pos.tolist() if start_pos is not None else [0] * (len(cq) - 1)
    for s in range(len(cq) - 1):
        for r in range(cq[s], cq[s + 1], rows_per_tile):
            last_key = sp[s] + min(r + rows_per_tile, cq[s + 1]) - cq[s]
            items.append((last_key, s, r))
    items.sort(key=lambda x: -x[0])
    return torch.tensor([(s, r) for _, s, r in items], dtype=torch.int32).reshape(-1, 2)


PREFILL_KT = 64          # keys per tile of the 32x32 prefill kernel (attention_prefill32.hip)


def prefill_split_plan(cu_q: torch.Tensor, rows_per_tile: int, start_pos, n_kv_heads: int,
                       num_cus: Optional[int] = None, min_chunk_tiles: int = 8):
    """Key-split work list for the varlen prefill kernel when its whole tiles would leave CUs idle
    (tensor-parallel shards: one or two KV heads per rank give ``tiles x Hkv`` << CUs, e.g. 28
    workgroups for a 1.8K-token prefill at tp 8). Returns None when the tiles alone fill half the
    chip; else ``(items [n, 5], cmap [m, 4], parts)``: items = (sequence, first row, first / end
    key tile of 64 keys, partial slot or -1), heaviest first; a tile longer than the chunk is cut
    into equal key ranges whose partial slots are consecutive and merged by the combine launch
    (cmap = sequence, first row, first slot, parts). Chunk = the tiles' total key work spread over
    ~2 workgroups per CU, at least ``min_chunk_tiles`` key tiles (partials cost a write + read
    of 128 floats per query row and head each)."""
    cq = cu_q.tolist()
    sp = start_pos.tolist() if start_pos is not None else [0] * (len(cq) - 1)
    tiles = []
    for s in range(len(cq) - 1):
        for r in range(cq[s], cq[s + 1], rows_per_tile):
            last_key = sp[s] + min(r + rows_per_tile, cq[s + 1]) - cq[s]
            tiles.append((s, r, (last_key + PREFILL_KT - 1) // PREFILL_KT))
    num_cus = device_cus() if num_cus is None else num_cus
    hkv = max(1, n_kv_heads)
    if not tiles or len(tiles) * hkv >= num_cus // 2:
        return None
    target = max(1, (2 * num_cus) // hkv)
    total = sum(t[2] for t in tiles)
    chunk = max(min_chunk_tiles, -(-total // target))
    items, cmap, p = [], [], 0
    for s, r, nkt in tiles:
        if nkt <= chunk:
            items.append((nkt, (s, r, 0, nkt, -1)))
            continue
        n = -(-nkt // chunk)
        per = -(-nkt // n)
        cmap.append((s, r, p, n))
        for j in range(n):
            tb = j * per
            te = min(nkt, tb + per)
            items.append((te - tb, (s, r, tb, te, p + j)))
        p += n
    if not cmap:
        return None
    items.sort(key=lambda x: -x[0])
    return (torch.tensor([it for _, it in items], dtype=torch.int32).reshape(-1, 5),
            torch.tensor(cmap, dtype=torch.int32).reshape(-1, 4), p)


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                      cu_q: torch.Tensor, start_pos: torch.Tensor, scale: float,
                      tile_map: Optional[torch.Tensor] = None, split=None) -> torch.Tensor:
    """``split``: a device-resident :func:`prefill_split_plan` ``(items, cmap, parts)`` — the
    key-split launch + its combine; ``tile_map`` otherwise (whole tiles)."""
    if _use_native(q):
        nat = native()
        out = torch.empty_like(q)
        if split is not None:
            items, cmap, parts = split
            hkv, D = k_cache.shape[1], q.shape[2]
            part_o = torch.empty(parts * hkv * 8 * 32 * D, dtype=torch.float32, device=q.device)
            part_ml = torch.empty(parts * hkv * 8 * 32 * 2, dtype=torch.float32, device=q.device)
            nat.prefill_attention_split(out, q, k_cache, v_cache, block_tables, cu_q, start_pos, items, cmap,
                                        part_o, part_ml, parts, scale)
            return out
        rows = nat.prefill_rows_per_tile(q.shape[1] // k_cache.shape[1], q.shape[2])
        if tile_map is None:
            tile_map = prefill_tile_map(cu_q.cpu(), rows, start_pos.cpu()).to(q.device)
        nat.prefill_attention(out, q, k_cache, v_cache, block_tables, cu_q, start_pos, tile_map, scale)
        return out
    return ref.prefill_attention(q, k_cache, v_cache, block_tables, cu_q.cpu(), start_pos.cpu(), scale)


PRO_PLAIN, PRO_NORM, PRO_NORM_ADD = 0, 1, 2
EPI_STORE, EPI_RESID, EPI_SWIGLU, EPI_ROPE = 0, 1, 2, 3


def shuffle_weight(W: torch.Tensor, gamma: Optional[torch.Tensor] = None, rope_heads: int = 0,
                   head_dim: int = 0, swiglu: bool = False) -> torch.Tensor:
    """Decode-weight copy in the MFMA fragment order of csrc/gemm_skinny.hip, with an RMSNorm
    weight ``gamma`` (over K) optionally folded in and, for a qkv weight used with
    :func:`skinny_gemm_rope`, the first ``rope_heads`` heads' rows pair-interleaved. ``swiglu``:
    W = [gate; up] for the SWIGLU epilogue, stored k-step-paired (one contiguous stream per wave).
    On CPU: the row-major ``W * gamma`` (rows permuted the same way; ``swiglu`` changes nothing)."""
    if _use_native(W):
        Ws = torch.empty_like(W)
        native().shuffle_weight(Ws, W.contiguous(), gamma, int(rope_heads), int(head_dim), bool(swiglu))
        return Ws
    return ref.fold_gamma(W, gamma, rope_heads, head_dim)


def kv_block_copy(k: torch.Tensor, v: torch.Tensor, src, dst) -> None:
    """K8: copy whole KV blocks ``src[i] -> dst[i]`` in every layer of both caches (``[L, NB, E]``)
    in one launch (csrc/kv_copy.hip); CPU: indexed copies."""
    if not src:
        return
    if _use_native(k):
        s_t = torch.tensor(list(src), dtype=torch.int32, device=k.device)
        d_t = torch.tensor(list(dst), dtype=torch.int32, device=k.device)
        native().kv_block_copy(k, v, s_t, d_t)
        return
    si, di = torch.tensor(list(src)), torch.tensor(list(dst))
    k[:, di] = k[:, si]
    v[:, di] = v[:, si]


def unshuffle_weight(Ws: torch.Tensor, rope_heads: int = 0, head_dim: int = 0, swiglu: bool = False,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-major weight back from a :func:`shuffle_weight` copy: the exact inverse permutation
    (a folded RMSNorm gamma stays folded). Lets a knight keep ONLY the shuffled weights resident
    and rebuild each prefill GEMM's row-major operand in a reused scratch buffer."""
    if out is None:
        out = torch.empty_like(Ws)
    if _use_native(Ws):
        native().unshuffle_weight(out, Ws, int(rope_heads), int(head_dim), bool(swiglu))
        return out
    if rope_heads:
        inv = torch.empty(Ws.shape[0], dtype=torch.long)
        inv[ref.rope_row_perm(Ws.shape[0], rope_heads, head_dim)] = torch.arange(Ws.shape[0])
        out.copy_(Ws[inv])
    else:
        out.copy_(Ws)
    return out


# split-K / CU-balanced skinny GEMM workspace: 256 tile counters + 528 floats per tile part, up
# to 1024 parts (split-K: T x S; balanced: 2 x (tile count mod CU count));
# csrc/gemm_skinny.hip splitk_parts / split_workspace_ints
SPLIT_WS_INTS = 256 + 1024 * (16 * 16 * 2 + 16)
SPLIT_K, SPLIT_BALANCE = 2, 1     # split_mode bits


def split_workspace(device) -> torch.Tensor:
    """Zeroed workspace for :func:`skinny_gemm` ``split_ws``. Launches on ONE stream may share it
    (its counters return to zero at the end of every call); concurrent launches must not."""
    return torch.zeros(SPLIT_WS_INTS, dtype=torch.int32, device=device)


def skinny_gemm(x: torch.Tensor, Ws: torch.Tensor, pro: int = PRO_PLAIN, epi: int = EPI_STORE,
                res: Optional[torch.Tensor] = None, eps: float = 1e-5, x2: Optional[torch.Tensor] = None,
                xout: Optional[torch.Tensor] = None, split_ws: Optional[torch.Tensor] = None,
                split_mode: int = SPLIT_K | SPLIT_BALANCE) -> Optional[torch.Tensor]:
    """Decode linear (M <= 16; up to 32 with the plain / norm prologues) on shuffled weights with fused RMSNorm prologue (gamma pre-folded)
    and residual / SwiGLU epilogue. Returns the output (None for RESID, which updates ``res``).
    ``PRO_NORM_ADD``: normalizes ``bf16(x + x2)`` and writes that sum to ``xout`` (TP decode).
    ``split_ws`` (:func:`split_workspace`) enables, per ``split_mode`` bit: ``SPLIT_K`` — fewer
    tiles than CUs (tensor-parallel shards): each tile's K range runs as S workgroups whose last
    arriver combines; ``SPLIT_BALANCE`` — tile count not a multiple of the CU count: the remainder
    tiles run as two K-halves so every CU streams the same bytes."""
    if _use_native(x):
        n = Ws.shape[0] // (2 if epi == EPI_SWIGLU else 1)
        out = torch.empty(x.shape[0], n, dtype=x.dtype, device=x.device) if epi != EPI_RESID else x
        native().skinny_gemm(out, x, Ws, pro, epi, res, eps, x2, xout, split_ws, int(split_mode))
        return None if epi == EPI_RESID else out
    return ref.skinny_gemm(x, Ws, pro, epi, res, eps, x2, xout)


def skinny_gemm_rope(x: torch.Tensor, Ws: torch.Tensor, pro: int, positions: torch.Tensor, cos_sin: torch.Tensor,
                     k_cache: torch.Tensor, v_cache: torch.Tensor, slots: torch.Tensor, n_heads: int,
                     n_kv_heads: int, head_dim: int, eps: float = 1e-5, x2: Optional[torch.Tensor] = None,
                     xout: Optional[torch.Tensor] = None, split_ws: Optional[torch.Tensor] = None,
                     split_mode: int = SPLIT_K | SPLIT_BALANCE, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode qkv projection (+ optional RMSNorm prologue) with RoPE and the paged K/V cache
    write fused into the epilogue; returns q [M, n_heads, head_dim]. ``Ws`` must come from
    ``shuffle_weight(Wqkv, gamma, rope_heads=n_heads + n_kv_heads, head_dim=head_dim)``.
    ``split_ws`` / ``split_mode``: as in :func:`skinny_gemm` (no balanced launch with ``PRO_NORM_ADD``).
    ``bias`` (Qwen2 q/k/v bias, added after the norm scale and before RoPE) must come from
    :func:`rope_bias` (fp32, the shuffled weight's column order)."""
    if _use_native(x):
        q = torch.empty(x.shape[0], n_heads, head_dim, dtype=x.dtype, device=x.device)
        native().skinny_gemm_rope(q, x, Ws, pro, positions, cos_sin, k_cache, v_cache, slots, n_heads, n_kv_heads,
                                  head_dim, eps, x2, xout, split_ws, int(split_mode), bias)
        return q
    return ref.skinny_gemm_rope(x, Ws, pro, positions, cos_sin, k_cache, v_cache, slots, n_heads, n_kv_heads,
                                head_dim, eps, x2, xout, bias)


def rope_bias(b: torch.Tensor, n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    """A q/k/v bias [(n_heads + 2 n_kv_heads) * head_dim] in the form :func:`skinny_gemm_rope` adds it."""
    return ref.rope_bias(b, n_heads + n_kv_heads, head_dim)


def decode_prep(slots: torch.Tensor, offsets: torch.Tensor, res: torch.Tensor, ids: torch.Tensor,
                positions: torch.Tensor, block_tables: torch.Tensor, embed: torch.Tensor, block_size: int) -> None:
    """Captured-step prologue (csrc/decode_step.hip): K/V slots, sampler offsets, embedding rows."""
    if _use_native(ids):
        native().decode_prep(slots, offsets, res, ids, positions, block_tables, embed, int(block_size))
        return
    ref.decode_prep(slots, offsets, res, ids, positions, block_tables, embed, block_size)


def paging_guard(block_tables: torch.Tensor, ctx_lens: torch.Tensor, positions: Optional[torch.Tensor],
                 slots: Optional[torch.Tensor], err: torch.Tensor, num_blocks: int, block_size: int) -> None:
    """Debug-mode device guard of the paging metadata (err[0] |= ref.PAGING_GUARD_CODES bits).

    Capturable: placed inside the decode hipGraph it validates the slots / lengths the graph
    advances on the device, which host-side asserts never see."""
    if _use_native(ctx_lens):
        native().paging_guard(block_tables, ctx_lens, positions, slots, err, int(num_blocks), int(block_size))
        return
    ref.paging_guard(block_tables, ctx_lens, positions, slots, err, num_blocks, block_size)


def paging_guard_message(code: int) -> str:
    return "; ".join(msg for bit, msg in ref.PAGING_GUARD_CODES.items() if code & bit) or "ok"


def decode_advance(out: torch.Tensor, ids: torch.Tensor, positions: torch.Tensor, ctx_lens: torch.Tensor,
                   step: torch.Tensor, nxt: torch.Tensor, prep=None) -> None:
    """Captured-step epilogue: record the sampled ids and advance positions / lengths / step.

    prep = (slots, offsets, res, block_tables, embed, block_size) also runs the NEXT step's
    decode_prep from the advanced ids / positions in the same launch."""
    if _use_native(ids):
        if prep is None:
            native().decode_advance(out, ids, positions, ctx_lens, step, nxt)
        else:
            slots, offsets, res, bt, embed, bs = prep
            native().decode_advance(out, ids, positions, ctx_lens, step, nxt, slots, offsets, res, bt, embed, int(bs))
        return
    ref.decode_advance(out, ids, positions, ctx_lens, step, nxt, prep)


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    if _use_native(x):
        out = torch.empty(*x.shape[:-1], x.shape[-1] // 2, dtype=x.dtype, device=x.device)
        native().silu_and_mul(out, x)
        return out
    return ref.silu_and_mul(x)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    if _use_native(x):
        out = torch.empty_like(x)
        native().gelu_tanh(out, x)
        return out
    return ref.gelu_tanh(x)


def sample_workspace(batch: int, device) -> torch.Tensor:
    """Zeroed K6 workspace for ``batch`` rows: its arrival tickets re-arm themselves after every
    launch, so one persistent workspace serves every replay of a captured step (no memset)."""
    return torch.zeros(native().sample_workspace_floats(batch), dtype=torch.float32, device=device)


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
           seeds: torch.Tensor, offsets: torch.Tensor, out: Optional[torch.Tensor] = None,
           ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-row ``offsets`` (int64, device-resident: the knight's position) keep hipGraph replays
    deterministic. ``ws``: a :func:`sample_workspace` (one is zero-allocated per call otherwise)."""
    if _use_native(logits):
        if out is None:
            out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
        nat = native()
        if ws is None:
            ws = sample_workspace(logits.shape[0], logits.device)
        nat.sample(out, logits, temperature, top_p, top_k, seeds, offsets, ws)
        return out
    return ref.sample(logits, temperature, top_p, top_k, seeds, offsets)


def sample_advance(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
                   seeds: torch.Tensor, offsets: torch.Tensor, ws: torch.Tensor, nxt: torch.Tensor,
                   out: torch.Tensor, ids: torch.Tensor, positions: torch.Tensor, ctx_lens: torch.Tensor,
                   step: torch.Tensor, slots: torch.Tensor, res: torch.Tensor, block_tables: torch.Tensor,
                   embed: torch.Tensor, block_size: int) -> torch.Tensor:
    """The captured decode step's K6 sampler fused with :func:`decode_advance` + the next step's
    :func:`decode_prep` (one launch): samples ``nxt`` from ``logits`` with the RNG ``offsets``, then
    records it in ``out[step]``, advances ids / positions / lengths / step and writes the next
    step's K/V slots, ``offsets`` and embedding rows."""
    if _use_native(logits):
        native().sample_advance(nxt, logits, temperature, top_p, top_k, seeds, offsets, ws, out, ids, positions,
                                ctx_lens, step, slots, res, block_tables, embed, int(block_size))
        return nxt
    nxt.copy_(ref.sample(logits, temperature, top_p, top_k, seeds, offsets))
    ref.decode_advance(out, ids, positions, ctx_lens, step, nxt, (slots, offsets, res, block_tables, embed,
                                                                  block_size))
    return nxt
