"""Torch-tensor front end of the C ABI (include/nrk.h).

Every op validates shapes / dtypes / devices on the host before it launches
(the kernels trust their arguments), runs on the current HIP stream, and
allocates its outputs and workspace with the torch caching allocator.
"""
from __future__ import annotations

import torch

from . import _lib

_P = _lib.P


def _stream():
    return _P(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return _P(t.data_ptr()) if t is not None else None


def _dev(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("nrk ops need device (cuda/HIP) tensors")
        if not t.is_contiguous():
            raise ValueError("nrk ops need contiguous tensors")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError("tensors on different devices")
    return dev


def _need(t, dtype, shape=None, name="tensor"):
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")


def _finite(t, name):
    """The screen kernels are built with -fno-honor-nans (Makefile): NaN / inf
    inputs would silently break their max chains, so the entry points that
    take outside vectors check them here (one reduction + sync)."""
    if t.numel() and not bool(torch.isfinite(t).all()):
        raise ValueError(f"{name} must be finite (NaN / inf found)")


# ------------------------------------------------------------------ tower --
def tt_user_fwd(user_table, item_table, uid, hist, hist_len, w0, b0, w1, b1, validate: bool = True, out=None):
    """YoutubeDNN user tower + re-normalisation (youtubednn_recaller.py:129-178, :467-470).
    ``validate`` checks hist_len against [0, T] (two device syncs); a caller
    that re-runs the tower on inputs it already validated (the bench's timed
    steps) may pass False.  ``out``: a preallocated fp32 [n, w1 rows] output
    (a pipelining caller's double buffer)."""
    _dev(user_table, item_table, uid, hist, hist_len, w0, b0, w1, b1)
    n, T = hist.shape
    D = user_table.shape[1]
    h0, h1 = w0.shape[0], w1.shape[0]
    _need(user_table, torch.float32, name="user_table")
    _need(item_table, torch.float32, (item_table.shape[0], D), "item_table")
    _need(uid, torch.int32, (n,), "uid")
    _need(hist, torch.int32, name="hist")
    _need(hist_len, torch.int32, (n,), "hist_len")
    _need(w0, torch.float32, (h0, 2 * D), "w0")
    _need(b0, torch.float32, (h0,), "b0")
    _need(w1, torch.float32, (h1, h0), "w1")
    _need(b1, torch.float32, (h1,), "b1")
    if validate and n and (int(hist_len.min()) < 0 or int(hist_len.max()) > T):
        raise ValueError("hist_len out of [0, T]")
    if out is None:
        out = torch.empty((n, h1), dtype=torch.float32, device=uid.device)
    else:
        _dev(out)
        _need(out, torch.float32, (n, h1), "out")
        if not out.is_contiguous():
            raise ValueError("out must be contiguous")
    _lib.call("nrk_tt_user_fwd", _ptr(user_table), user_table.shape[0], _ptr(item_table),
              item_table.shape[0], D, _ptr(uid), _ptr(hist), _ptr(hist_len), n, T,
              _ptr(w0), _ptr(b0), h0, _ptr(w1), _ptr(b1), h1, _ptr(out), _stream())
    return out


def tt_user_fwd_layers(user_table, item_table, uid, hist, hist_len, layers):
    """The user tower at any depth (youtubednn_recaller.py:105-112):
    ``layers`` = [(W_l [w_l, in_l], b_l [w_l]), ...] fp32 device tensors, the
    last width equal to the embedding dim."""
    import ctypes

    _dev(user_table, item_table, uid, hist, hist_len, *[t for wb in layers for t in wb])
    n, T = hist.shape
    D = user_table.shape[1]
    _need(user_table, torch.float32, name="user_table")
    _need(item_table, torch.float32, (item_table.shape[0], D), "item_table")
    _need(uid, torch.int32, (n,), "uid")
    _need(hist, torch.int32, name="hist")
    _need(hist_len, torch.int32, (n,), "hist_len")
    widths, packed, fan_in = [], [], 2 * D
    for l, (w, b) in enumerate(layers):
        _need(w, torch.float32, (w.shape[0], fan_in), f"W{l}")
        _need(b, torch.float32, (w.shape[0],), f"b{l}")
        widths.append(int(w.shape[0]))
        packed += [w.reshape(-1), b]
        fan_in = w.shape[0]
    if n and (int(hist_len.min()) < 0 or int(hist_len.max()) > T):
        raise ValueError("hist_len out of [0, T]")
    wts = torch.cat(packed).contiguous()
    out = torch.empty((n, D), dtype=torch.float32, device=uid.device)
    wv = (ctypes.c_int * len(widths))(*widths)
    _lib.call("nrk_tt_user_fwd_layers", _ptr(user_table), user_table.shape[0], _ptr(item_table),
              item_table.shape[0], D, _ptr(uid), _ptr(hist), _ptr(hist_len), n, T, _ptr(wts), len(widths),
              ctypes.cast(wv, _P), _ptr(out), _stream())
    return out


def tt_item_fwd(item_table, ids):
    """get_item_embedding + re-normalisation (youtubednn_recaller.py:184-188, :485-489)."""
    _dev(item_table, ids)
    _need(item_table, torch.float32, name="item_table")
    _need(ids, torch.int32, name="ids")
    n, D = ids.shape[0], item_table.shape[1]
    out = torch.empty((n, D), dtype=torch.float32, device=ids.device)
    _lib.call("nrk_tt_item_fwd", _ptr(item_table), item_table.shape[0], D, _ptr(ids), n,
              _ptr(out), _stream())
    return out


# ------------------------------------------------------------------ top-k --
IP_KFAST = 128   # k on the MFMA screen path (csrc/ip_topk.hip); larger k takes the exact path
IP_KMAX = 2048   # largest k compiled
CF_TOPK_MAX = 2048  # nrk_itemcf_topn / nrk_itemcf_recall (register path <= 64, LDS path above)


class Catalog:
    """The search index: fp32 rows (kept for exact rescoring) + a scaled fp16
    copy packed in MFMA fragment order.  = faiss.IndexFlatIP(d).add(items);
    rejects NaN / inf rows."""

    def __init__(self, items: torch.Tensor):
        _dev(items)
        _need(items, torch.float32, name="items")
        if items.dim() != 2 or not (1 <= items.shape[1] <= 256):
            raise ValueError("items must be [n, d] with 1 <= d <= 256")
        _finite(items, "items")
        self.items = items
        self.n, self.d = items.shape
        nbytes = _lib.lib().nrk_ip_catalog_bytes(self.n, self.d)
        self.packed = torch.empty(nbytes, dtype=torch.uint8, device=items.device)
        _lib.call("nrk_ip_catalog_build", _ptr(items), self.n, self.d, _ptr(self.packed), _stream())

    @property
    def ntotal(self):
        return self.n


def ip_topk(users, catalog: Catalog, k: int, row_offset: int = 0, exact: bool = False, workspace=None,
            check_finite: bool = True):
    """Exact top-k rows per user (scores f32 [n,k], rows i32 [n,k] (+ fp64)).
    ``check_finite`` rejects NaN / inf users (one device sync); the split
    screen entry points (ip_topk_screen*, the bench / catalog-sharded path)
    leave that to the caller."""
    _dev(users, catalog.items)
    _need(users, torch.float32, name="users")
    if users.dim() != 2 or users.shape[1] != catalog.d:
        raise ValueError(f"users must be [n, {catalog.d}]")
    if check_finite:
        _finite(users, "users")
    if not (1 <= k <= IP_KMAX):
        raise ValueError(f"k must be in [1, {IP_KMAX}]")
    n = users.shape[0]
    dev = users.device
    s = torch.empty((n, k), dtype=torch.float32, device=dev)
    r = torch.empty((n, k), dtype=torch.int32, device=dev)
    e = torch.empty((n, k), dtype=torch.float64, device=dev) if exact else None
    ws_bytes = _lib.lib().nrk_ip_topk_workspace_bytes(n, catalog.n, catalog.d, k)
    if workspace is None or workspace.numel() < ws_bytes:
        workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    _lib.call("nrk_ip_topk", _ptr(users), n, _ptr(catalog.items), _ptr(catalog.packed), catalog.n,
              catalog.d, k, int(row_offset), _ptr(s), _ptr(r), _ptr(e), _ptr(workspace),
              workspace.numel(), _stream())
    return (s, r, e) if exact else (s, r)


def ip_topk_workspace(n_users, catalog: Catalog, k, device):
    nb = _lib.lib().nrk_ip_topk_workspace_bytes(n_users, catalog.n, catalog.d, k)
    return torch.empty(nb, dtype=torch.uint8, device=device)


def topk_merge(exact_lists, row_lists, k_out):
    """Merge [G, n, k_in] per-shard lists (fp64 scores + global rows)."""
    _dev(exact_lists, row_lists)
    _need(exact_lists, torch.float64, name="exact_lists")
    _need(row_lists, torch.int32, tuple(exact_lists.shape), "row_lists")
    G, n, k_in = exact_lists.shape
    if G * k_in > 1024 or k_out > G * k_in:
        raise ValueError("need G*k_in <= 1024 and k_out <= G*k_in")
    dev = exact_lists.device
    s = torch.empty((n, k_out), dtype=torch.float32, device=dev)
    r = torch.empty((n, k_out), dtype=torch.int32, device=dev)
    e = torch.empty((n, k_out), dtype=torch.float64, device=dev)
    _lib.call("nrk_topk_merge", _ptr(exact_lists), _ptr(row_lists), G, n * k_in, n, k_in, k_out,
              _ptr(s), _ptr(r), _ptr(e), _stream())
    return s, r, e


def ip_topk_screen(users, catalog: Catalog, k: int, workspace):
    """Phase 1 of ip_topk (fp16 MFMA scan -> candidate band in ``workspace``).
    ``users`` must be finite (not checked here: the hot path)."""
    _dev(users, workspace)
    n = users.shape[0]
    _lib.call("nrk_ip_topk_screen", _ptr(users), n, _ptr(catalog.packed), catalog.n, catalog.d, k,
              _ptr(workspace), workspace.numel(), _stream())


def ip_topk_scan(users, catalog: Catalog, k: int, workspace):
    """ip_topk_screen's first launch alone: the fp16 MFMA scan (appends)."""
    _dev(users, workspace)
    _lib.call("nrk_ip_topk_scan", _ptr(users), users.shape[0], _ptr(catalog.packed), catalog.n, catalog.d, k,
              _ptr(workspace), workspace.numel(), _stream())


def ip_topk_select(users, catalog: Catalog, k: int, workspace):
    """ip_topk_screen's second launch alone: the per-user select (band)."""
    _dev(users, workspace)
    _lib.call("nrk_ip_topk_select", _ptr(users), users.shape[0], _ptr(catalog.packed), catalog.n, catalog.d, k,
              _ptr(workspace), workspace.numel(), _stream())


def ip_topk_finish(users, catalog: Catalog, k: int, workspace, out_scores, out_rows,
                   out_exact=None, row_offset: int = 0):
    """Phase 2 of ip_topk (exact rescoring + ordering) into preallocated outputs."""
    _dev(users, workspace, out_scores, out_rows, out_exact)
    n = users.shape[0]
    _lib.call("nrk_ip_topk_finish", _ptr(users), n, _ptr(catalog.items), _ptr(catalog.packed), catalog.n, catalog.d, k,
              int(row_offset), _ptr(out_scores), _ptr(out_rows), _ptr(out_exact), _ptr(workspace),
              workspace.numel(), _stream())


def ip_topk_bound(users, catalog: Catalog, k: int, m: int, workspace):
    """After ip_topk_screen (same k): per user the m largest exact lower
    bounds of this shard (fp32 [n, m], descending, -inf padded), each
    bounding a distinct item's exact score."""
    _dev(users, workspace)
    n = users.shape[0]
    out = torch.empty((n, m), dtype=torch.float32, device=users.device)
    _lib.call("nrk_ip_topk_bound", _ptr(users), n, _ptr(catalog.packed), catalog.n, catalog.d, int(k), int(m),
              _ptr(out),
              _ptr(workspace), workspace.numel(), _stream())
    return out


def ip_topk_tile_blocks(d: int) -> int:
    """32-item blocks per screen tile (shard ranges start on a tile):
    nrk_ip_topk_tile_blocks, the scan's own constant (no device work)."""
    tb = _lib.lib().nrk_ip_topk_tile_blocks(int(d))
    if tb <= 0:
        raise ValueError(f"dim must be in [1, 256], got {d}")
    return tb


def ip_topk_shard_screen(users, catalog: Catalog, k: int, blk_lo: int, blk_hi: int, m: int, workspace):
    """Config-4 shard, select-free: the scan of the blocks [blk_lo, blk_hi)
    for every user + per user the m largest appended maxima as exact lower
    bounds (fp32 [n, m], descending, -inf padded)."""
    _dev(users, workspace)
    n = users.shape[0]
    out = torch.empty((n, m), dtype=torch.float32, device=users.device)
    _lib.call("nrk_ip_topk_shard_screen", _ptr(users), n, _ptr(catalog.packed), catalog.n, catalog.d, int(k),
              int(blk_lo), int(blk_hi), int(m), _ptr(out), _ptr(workspace), workspace.numel(), _stream())
    return out


IP_X_CAP = 32  # band half-block ids per user and shard in the fixed-slot exchange (4 B each)


def ip_topk_shard_band(n_users, catalog: Catalog, k: int, bounds, workspace, x_cap: int = IP_X_CAP):
    """After ip_topk_shard_screen and the all_gather of every shard's bounds
    (``bounds`` [n_lists, n_users, m] f32, or None): cut = max(own list bound
    - 2 eps, k-th largest bound - eps), the half-blocks >= cut packed: (cnt
    int32 [n] (-1 = more than x_cap: exact path), ids int32 [n, x_cap]
    (global half-block ids)); the cut goes to ucut."""
    cap = int(x_cap)
    dev = workspace.device
    cnt = torch.empty(n_users, dtype=torch.int32, device=dev)
    ent = torch.empty((n_users, cap), dtype=torch.int32, device=dev)
    nl, m = (0, 1) if bounds is None else (bounds.shape[0], bounds.shape[2])
    if bounds is not None:
        _dev(bounds, workspace)
        _need(bounds, torch.float32, (nl, n_users, m), "bounds")
    _lib.call("nrk_ip_topk_shard_band", n_users, catalog.n, catalog.d, int(k), _ptr(bounds), nl, m, cap,
              _ptr(workspace), workspace.numel(), _ptr(ent), _ptr(cnt), _stream())
    return cnt, ent


def ip_topk_refine_x(users, catalog: Catalog, k: int, src_cnt, src_ent, ucut, ovf=None, row_offset: int = 0,
                     workspace=None):
    """The config-4 owner's exact refine over the fixed-slot exchange:
    ``src_ent`` int32 [n_src, src_users, x_cap] (source s's band half-block
    ids of user u), ``src_cnt`` int32 [n_src, src_users] (-1: exact path), users
    [n <= src_users, D].  Returns (scores f32 [n, k], rows i32 [n, k],
    exact f64 [n, k])."""
    _dev(users, src_cnt, src_ent, ucut, ovf)
    n = users.shape[0]
    ns, su, x = src_ent.shape
    _need(src_ent, torch.int32, name="src_ent")
    _need(src_cnt, torch.int32, (ns, su), "src_cnt")
    if su < n:
        raise ValueError("src_users must cover the users")
    dev = users.device
    s = torch.empty((n, k), dtype=torch.float32, device=dev)
    r = torch.empty((n, k), dtype=torch.int32, device=dev)
    e = torch.empty((n, k), dtype=torch.float64, device=dev)
    nb = _lib.lib().nrk_ip_topk_workspace_bytes(n, catalog.n, catalog.d, k)
    if workspace is None or workspace.numel() < nb:
        workspace = torch.empty(nb, dtype=torch.uint8, device=dev)
    _lib.call("nrk_ip_topk_refine_x", _ptr(users), n, _ptr(catalog.items), _ptr(catalog.packed), catalog.n,
              catalog.d, int(k), int(row_offset), _ptr(src_ent), ns, su, x, _ptr(src_cnt), _ptr(ucut), _ptr(ovf),
              _ptr(s), _ptr(r), _ptr(e), _ptr(workspace), workspace.numel(), _stream())
    return s, r, e


def ip_topk_ucut(workspace, n_users):
    """The per-user (cut, eps) float32 [n, 2] of a top-k workspace (ip_ws_layout: after the 256-B header)."""
    return workspace[256: 256 + 8 * n_users].view(torch.float32).view(n_users, 2)


def ip_topk_apply_bound(bounds, k: int, workspace):
    """bounds [n_lists, n, m] fp32 (every shard's ip_topk_bound): raise this
    shard's refine cut to the k-th largest of each user's n_lists * m values."""
    _dev(bounds, workspace)
    _need(bounds, torch.float32, name="bounds")
    if bounds.dim() != 3:
        raise ValueError("bounds must be [n_lists, n_users, m]")
    L, n, m = bounds.shape
    _lib.call("nrk_ip_topk_apply_bound", n, _ptr(bounds), L, m, int(k), _ptr(workspace), workspace.numel(),
              _stream())


def row_normalize(x, norms=False):
    """x / ||x|| per row, bit-identical to numpy float32 (similarity/embedding.py:41)."""
    _dev(x)
    _need(x, torch.float32, name="x")
    if x.dim() != 2 or not (1 <= x.shape[1] <= 256):
        raise ValueError("x must be [n, d] with 1 <= d <= 256")
    n, d = x.shape
    out = torch.empty_like(x)
    nr = torch.empty(n, dtype=torch.float32, device=x.device) if norms else None
    _lib.call("nrk_row_normalize", _ptr(x), n, d, _ptr(out), _ptr(nr), _stream())
    return (out, nr) if norms else out


# -------------------------------------------------------------------- DIN --
DIN_KERNEL_ITEM_FEATS = (1, 2, 4, 8)  # item-feature counts the attention kernels are instantiated for


class DinParams:
    """Device-resident DIN weights in kernel layout (DINModel state_dict,
    DIN.py:133-212): concatenated embedding table (fp32 or bf16 storage),
    per-feature row offsets, prepared attention matrices and the MLP.

    Any embedding width D (``din_embedding_dim``, config.py:115; the
    state_dict's table width) and any item-feature count up to 8 32-wide
    features: the kernels read 32-wide VIRTUAL features.  Every table is
    zero-padded to m = ceil(D / 32) * 32 columns and viewed as [m * vocab, 32]
    (feature f's index i -> virtual indices m i + h), att_w0 / mlp_w0 get
    zero columns at the padded positions, and the item features are padded
    with a shared all-zero row up to 1, 2, 4 or 8 -- every extra product is
    an exact 0, so the results are those of the D-wide model.  ``n_user`` /
    ``n_item`` / ``n_ctx`` / ``vocab`` describe the caller's features;
    ``kn_*`` the kernel's (include/nrk.h, nrk_din_remap_index)."""

    def __init__(self, state_dict, user_feats, item_feats, ctx_feats, table_dtype="fp32",
                 device="cuda"):
        import numpy as np

        def arr(k):
            v = state_dict[k]
            v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
            return np.ascontiguousarray(v, dtype=np.float32)

        user_feats, item_feats, ctx_feats = list(user_feats), list(item_feats), list(ctx_feats)
        groups = ([("user_profile_embedding_dict", f) for f in user_feats]
                  + [("item_embedding_dict", f) for f in item_feats]
                  + [("context_embedding_dict", f) for f in ctx_feats])
        tabs = [arr(f"{g}.{f}.weight") for g, f in groups]
        if not tabs or not item_feats or not user_feats:
            raise ValueError("DIN needs at least one user and one item feature")
        D = tabs[0].shape[1]
        if any(t.ndim != 2 or t.shape[1] != D for t in tabs):
            raise ValueError("every embedding table must have the same width (din_embedding_dim)")
        m = -(-D // 32)
        Fu, Fi, Fc = len(user_feats), len(item_feats), len(ctx_feats)
        niv = m * Fi
        kni = next((n for n in DIN_KERNEL_ITEM_FEATS if n >= niv), None)
        if kni is None:
            raise NotImplementedError(f"DIN item features x ceil(dim / 32) must be <= 8, got {Fi} x {m}")
        self.dim, self.m = D, m
        self.n_user, self.n_item, self.n_ctx = Fu, Fi, Fc
        self.vocab = [t.shape[0] for t in tabs]
        self.kn_user, self.kn_item, self.kn_ctx = m * Fu, kni, m * Fc

        def virt(t):  # [v, D] -> [m v, 32], zero-padded columns
            if D == 32 * m:
                return t.reshape(-1, 32)
            tp = np.zeros((t.shape[0], 32 * m), np.float32)
            tp[:, :D] = t
            return tp.reshape(-1, 32)

        vt = [virt(t) for t in tabs]
        pieces = vt[:Fu] + vt[Fu:Fu + Fi] + ([np.zeros((1, 32), np.float32)] if kni > niv else []) + vt[Fu + Fi:]
        starts = np.cumsum([0] + [pc.shape[0] for pc in pieces[:-1]]).astype(np.int64)
        fb = list(starts[:Fu + Fi]) + list(starts[Fu + Fi + (1 if kni > niv else 0):])  # per caller feature
        zero_row = int(starts[Fu + Fi]) if kni > niv else 0
        # virtual feature (f, hh) of a caller feature f: row fb[f] + hh + m i for caller
        # index i -- base fb[f] + hh, virtual index m i -- so caller index 0 (the
        # collate's padding) stays virtual index 0 in every half, which is what the
        # position-major plan's padding test (mask 0, every index 0) and its pad row
        # (row 0 of each feature) assume (with index m i + hh no padding
        # row of a D > 32 model was ever recognised)
        base = ([fb[f] + hh for f in range(Fu) for hh in range(m)]
                + [fb[Fu + f] + hh for f in range(Fi) for hh in range(m)] + [zero_row] * (kni - niv)
                + [fb[Fu + Fi + f] + hh for f in range(Fc) for hh in range(m)])
        table = torch.from_numpy(np.concatenate(pieces, 0))
        _finite(table, "DIN embedding tables")
        if table_dtype == "bf16":
            self.table = table.to(torch.bfloat16).to(device).contiguous()
            self.table_code = 1
        elif table_dtype == "fp32":
            self.table = table.to(device).contiguous()
            self.table_code = 0
        else:
            raise ValueError("table_dtype must be 'fp32' or 'bf16'")
        self.row_base = torch.from_numpy(np.asarray(base, np.int64)).to(device)

        # index maps to the virtual layout (None: identity, no remap launch)
        def idx_map(F, pad_to):
            src = [f for f in range(F) for _ in range(m)] + [-1] * (pad_to - m * F)
            mul = [m] * (m * F) + [0] * (pad_to - m * F)
            add = [0] * pad_to
            return torch.tensor([src, mul, add], dtype=torch.int32).to(device).contiguous()

        self.map_user = None if m == 1 else idx_map(Fu, m * Fu)
        self.map_item = None if m == 1 and kni == Fi else idx_map(Fi, kni)
        self.map_ctx = None if m == 1 or Fc == 0 else idx_map(Fc, m * Fc)

        d = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device).contiguous()  # noqa: E731
        aw0 = arr("activation_unit.mlp.0.weight")
        w0 = arr("mlp.0.weight")
        if aw0.shape != (36, 4 * Fi * D) or w0.shape[1] != D * (Fu + Fc + 2 * Fi):
            raise ValueError("state_dict shapes do not match the feature lists")

        def expand(w, F, pad_to):  # [rows, F D] -> [rows, pad_to * 32]
            x = np.zeros((w.shape[0], F, 32 * m), np.float32)
            x[:, :, :D] = w.reshape(w.shape[0], F, D)
            x = x.reshape(w.shape[0], F * m * 32)
            if pad_to * 32 > x.shape[1]:
                x = np.concatenate([x, np.zeros((w.shape[0], pad_to * 32 - x.shape[1]), np.float32)], 1)
            return x

        self.att_w0 = d(np.concatenate([expand(aw0[:, q * Fi * D:(q + 1) * Fi * D], Fi, kni) for q in range(4)], 1))
        cuts = np.cumsum([0, Fu * D, Fc * D, Fi * D, Fi * D])
        segs = [(0, Fu, m * Fu), (1, Fc, m * Fc), (2, Fi, kni), (3, Fi, kni)]
        self.mlp_w0 = d(np.concatenate([expand(w0[:, cuts[i]:cuts[i + 1]], F, pt) for i, F, pt in segs], 1))
        self.att_b0 = d(arr("activation_unit.mlp.0.bias"))
        self.att_w1 = d(arr("activation_unit.mlp.2.weight").reshape(-1))
        self.att_b1 = d(arr("activation_unit.mlp.2.bias"))
        self.mlp_b0 = d(arr("mlp.0.bias"))
        self.mlp_w1, self.mlp_b1 = d(arr("mlp.2.weight")), d(arr("mlp.2.bias"))
        self.mlp_w2 = d(arr("mlp.4.weight").reshape(-1))
        self.mlp_b2 = d(arr("mlp.4.bias"))
        for name in ("att_w0", "att_b0", "att_w1", "att_b1", "mlp_w0", "mlp_b0", "mlp_w1", "mlp_b1", "mlp_w2",
                     "mlp_b2"):
            _finite(getattr(self, name), f"DIN weight {name}")
        self.h1, self.h2 = self.mlp_w0.shape[0], self.mlp_w1.shape[0]
        if self.mlp_w1.shape[1] != self.h1 or self.mlp_w2.numel() != self.h2 or self.att_w1.numel() != 36:
            raise ValueError("state_dict shapes do not match the feature lists")
        nb = _lib.lib().nrk_din_prep_bytes(self.kn_item, self.table.shape[0])
        self.prep = torch.empty(nb, dtype=torch.uint8, device=device)
        _lib.call("nrk_din_prepare", _ptr(self.att_w0), self.kn_item, _ptr(self.table), self.table_code,
                  self.table.shape[0], _ptr(self.prep), _stream())

    def kernel_indices(self, user, item, hist, ctx):
        """Caller index tensors -> the kernel's virtual-feature layout
        (nrk_din_remap_index); identity for 32-wide models with 1/2/4/8 item
        features."""
        def remap(t, mp, f_in):
            if mp is None:
                return t
            rows = t.numel() // f_in
            out = torch.empty(t.shape[:-1] + (mp.shape[1],), dtype=torch.int32, device=t.device)
            _lib.call("nrk_din_remap_index", _ptr(t), rows, f_in, _ptr(mp), mp.shape[1], _ptr(out), _stream())
            return out

        return (remap(user, self.map_user, self.n_user), remap(item, self.map_item, self.n_item),
                remap(hist, self.map_item, self.n_item), remap(ctx, self.map_ctx, self.n_ctx))


def din_validate(p: DinParams, user, item, hist, ctx):
    """Raise ValueError if any index falls outside its embedding table (the
    kernels gather without bounds checks)."""
    for t, off in ((user, 0), (item, p.n_user), (ctx, p.n_user + p.n_item)):
        if t.numel():
            mx = t.reshape(-1, t.shape[-1]).amax(0).cpu().tolist()
            mn = int(t.min())
            if mn < 0 or any(m >= p.vocab[off + f] for f, m in enumerate(mx)):
                raise ValueError("feature index out of its embedding table")
    if hist.numel():
        mx = hist.reshape(-1, p.n_item).amax(0).cpu().tolist()
        if int(hist.min()) < 0 or any(m >= p.vocab[p.n_user + f] for f, m in enumerate(mx)):
            raise ValueError("history index out of its embedding table")


def _din_seg(B, batch_size):
    S = B if batch_size is None or batch_size >= B else int(batch_size)
    if S < B and S % 64:
        raise ValueError("batch_size must be a multiple of 64 when the samples span several batches")
    if S == B and B < 2:
        raise ValueError("batch must be >= 2 (Dice uses the batch std; B = 1 is NaN in the reference)")
    return S


def din_forward(p: DinParams, user, item, hist, ctx, mask, logits=False, workspace=None,
                out=None, validate=True, batch_size=None):
    """DIN scores of B samples: int32 index tensors user [B,Fu], item [B,Fi],
    hist [B,T,Fi], ctx [B,Fc], mask [B,T] f32 -> probs [B] (+ logits).
    ``batch_size=None``: the B samples are one Dice batch (B >= 2).
    Otherwise they are scored as consecutive batches of ``batch_size`` (a
    multiple of 64), each with its own Dice statistics -- DINRanker.predict's
    loop (DIN.py:1245-1283) in one call; a trailing batch of one row is NaN
    as in the reference.
    ``validate=False`` skips the host-side index range check (one device sync)
    for callers that validated the resident index tensors once up front."""
    _dev(user, item, hist, ctx, mask)
    B, T = mask.shape
    S = _din_seg(B, batch_size)
    _need(user, torch.int32, (B, p.n_user), "user")
    _need(item, torch.int32, (B, p.n_item), "item")
    _need(hist, torch.int32, (B, T, p.n_item), "hist")
    _need(ctx, torch.int32, (B, p.n_ctx), "ctx")
    _need(mask, torch.float32, (B, T), "mask")
    if validate:
        din_validate(p, user, item, hist, ctx)
    user, item, hist, ctx = p.kernel_indices(user, item, hist, ctx)
    if out is not None:
        _need(out, torch.float32, (B,), "out")
        probs = out
    else:
        probs = torch.empty(B, dtype=torch.float32, device=mask.device)
    lg = torch.empty(B, dtype=torch.float32, device=mask.device) if logits else None
    nb = _lib.lib().nrk_din_segments_workspace_bytes(B, S, T, p.kn_user, p.kn_item, p.kn_ctx, p.h1, p.h2)
    if workspace is None or workspace.numel() < nb:
        workspace = torch.empty(nb, dtype=torch.uint8, device=mask.device)
    _lib.call("nrk_din_forward_segments", _ptr(p.table), p.table_code, _ptr(p.row_base), p.kn_user,
              p.kn_item, p.kn_ctx, _ptr(user), _ptr(item), _ptr(hist), _ptr(ctx), _ptr(mask), B, S, T,
              _ptr(p.prep), _ptr(p.att_b0), _ptr(p.att_w1), _ptr(p.att_b1), _ptr(p.mlp_w0),
              _ptr(p.mlp_b0), p.h1, _ptr(p.mlp_w1), _ptr(p.mlp_b1), p.h2, _ptr(p.mlp_w2),
              _ptr(p.mlp_b2), _ptr(probs), _ptr(lg), _ptr(workspace), workspace.numel(), _stream())
    if S < B and B % S == 1:  # trailing batch of one row: std undefined -> NaN (reference)
        probs[B - 1] = float("nan")
        if lg is not None:
            lg[B - 1] = float("nan")
    return (probs, lg) if logits else probs


def din_workspace(p: DinParams, B, T, device, batch_size=None):
    S = _din_seg(B, batch_size)
    nb = _lib.lib().nrk_din_segments_workspace_bytes(B, S, T, p.kn_user, p.kn_item, p.kn_ctx, p.h1, p.h2)
    return torch.empty(nb, dtype=torch.uint8, device=device)


# ----------------------------------------------------------------- itemcf --
class ItemCFSim:
    """Device result of nrk_itemcf_sim: one entry per distinct (i, j), sorted
    by (i, j), dense item ids.  ``first`` is the entry's first-encounter slot
    (the reference's dict insertion order); ``cnt`` the per-item click count."""

    def __init__(self, i, j, v, first, cnt, n_items):
        self.i, self.j, self.v, self.first, self.cnt = i, j, v, first, cnt
        self.n_items = n_items

    def row_offsets(self):
        """CSR offsets over dense item rows (entries are sorted by i)."""
        off = torch.empty(self.n_items + 1, dtype=torch.int64, device=self.i.device)
        _lib.call("nrk_itemcf_row_offsets", _ptr(self.i), self.i.numel(), self.n_items, _ptr(off), _stream())
        return off


def itemcf_sim(offsets, items, ts, created, n_items, loc_alpha=1.0, loc_alpha_rev=0.7,
               loc_beta=0.9, time_alpha=0.7, created_alpha=0.8):
    """ItemCF similarity (item_cf.py:17-89) over user click lists in CSR:
    offsets int64 [U+1], items int32 dense ids [N], ts int64 ms [N], created
    float64 per dense item [n_items]."""
    _dev(offsets, items, ts, created)
    _need(offsets, torch.int64, name="offsets")
    _need(items, torch.int32, (items.numel(),), "items")
    _need(ts, torch.int64, (items.numel(),), "ts")
    _need(created, torch.float64, (n_items,), "created")
    if offsets.dim() != 1 or offsets.numel() < 1:
        raise ValueError("offsets must be 1-D with n_users + 1 entries")
    n_users = offsets.numel() - 1
    dev = offsets.device
    if items.numel():
        if int(items.min()) < 0 or int(items.max()) >= n_items:
            raise ValueError("item id out of [0, n_items)")
    if int(offsets[0]) != 0 or int(offsets[-1]) != items.numel() or bool((offsets[1:] < offsets[:-1]).any()):
        raise ValueError("offsets must be non-decreasing from 0 to len(items)")
    pair_off = torch.empty(n_users + 1, dtype=torch.int64, device=dev)
    _lib.call("nrk_itemcf_pair_offsets", _ptr(offsets), n_users, _ptr(pair_off), _stream())
    n_pairs = int(pair_off[-1])
    cap = max(n_pairs, 1)
    oi = torch.empty(cap, dtype=torch.int32, device=dev)
    oj = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    of = torch.empty(cap, dtype=torch.int64, device=dev)
    on = torch.zeros(1, dtype=torch.int64, device=dev)
    cnt = torch.empty(n_items, dtype=torch.int64, device=dev)
    nb = _lib.lib().nrk_itemcf_workspace_bytes(n_pairs, n_items)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    _lib.call("nrk_itemcf_sim", _ptr(offsets), n_users, _ptr(items), _ptr(ts), _ptr(created),
              n_items, _ptr(pair_off), n_pairs, float(loc_alpha), float(loc_alpha_rev),
              float(loc_beta), float(time_alpha), float(created_alpha), _ptr(oi), _ptr(oj),
              _ptr(ov), _ptr(of), _ptr(on), _ptr(cnt), _ptr(ws), nb, _stream())
    n = int(on.item())
    return ItemCFSim(oi[:n], oj[:n], ov[:n], of[:n], cnt, n_items)


def itemcf_topn(row_off, cols, vals, first, topn=20):
    """Per-row top-n by (score desc, first asc) -- the reference's stable
    ``sorted(..., reverse=True)[:topn]`` (itemcf_recaller.py:41-54).
    Returns (cols [R, topn] int32 -1 padded, vals [R, topn] f64, cnt [R])."""
    if not (1 <= topn <= CF_TOPK_MAX):
        raise NotImplementedError(f"topn must be in [1, {CF_TOPK_MAX}]")
    _dev(row_off, cols, vals, first)
    _need(row_off, torch.int64, name="row_off")
    _need(cols, torch.int32, name="cols")
    _need(vals, torch.float64, (cols.numel(),), "vals")
    _need(first, torch.int64, (cols.numel(),), "first")
    n_rows = row_off.numel() - 1
    dev = row_off.device
    oc = torch.empty((n_rows, topn), dtype=torch.int32, device=dev)
    ov = torch.empty((n_rows, topn), dtype=torch.float64, device=dev)
    cnt = torch.empty(n_rows, dtype=torch.int32, device=dev)
    _lib.call("nrk_itemcf_topn", _ptr(row_off), n_rows, _ptr(cols), _ptr(vals), _ptr(first), int(topn),
              _ptr(oc), _ptr(ov), _ptr(cnt), _stream())
    return oc, ov, cnt


def itemcf_recall(q_slot, offsets, items, nbr_cols, nbr_vals, nbr_cnt, created, hot, topk,
                  loc_beta=0.9, created_alpha=0.8, emb_cols=None, emb_vals=None, emb_cnt=None):
    """ItemCFRecaller.recall (itemcf_recaller.py:56-129) for every query user at
    once.  Dense ids: q_slot [Q] int64 (CSR row or -1 = unknown user),
    offsets/items = the user_item_time_dict CSR, nbr_* = per-item top-n
    neighbours [I, topn] (itemcf_topn), created [I] f64, hot [H] int32,
    optional emb_* [I, ke] content-weight neighbours.  Returns (items [Q, topk]
    int32 -1 padded, scores [Q, topk] f64, src [Q, topk] int32 (0 candidate,
    1 hot fill, 2 cold start), cnt [Q] int32)."""
    _dev(q_slot, offsets, items, nbr_cols, nbr_vals, nbr_cnt, created, hot, emb_cols, emb_vals, emb_cnt)
    _need(q_slot, torch.int64, name="q_slot")
    _need(offsets, torch.int64, name="offsets")
    _need(items, torch.int32, name="items")
    n_items, topn = nbr_cols.shape
    _need(nbr_cols, torch.int32, name="nbr_cols")
    _need(nbr_vals, torch.float64, (n_items, topn), "nbr_vals")
    _need(nbr_cnt, torch.int32, (n_items,), "nbr_cnt")
    _need(created, torch.float64, (n_items,), "created")
    _need(hot, torch.int32, name="hot")
    ke = 0
    if emb_cols is not None:
        ke = emb_cols.shape[1]
        _need(emb_cols, torch.int32, (n_items, ke), "emb_cols")
        _need(emb_vals, torch.float64, (n_items, ke), "emb_vals")
        _need(emb_cnt, torch.int32, (n_items,), "emb_cnt")
    if not (1 <= topk <= CF_TOPK_MAX):
        raise NotImplementedError(f"topk must be in [1, {CF_TOPK_MAX}]")
    nq = q_slot.numel()
    dev = q_slot.device
    cand_off = torch.empty(nq + 1, dtype=torch.int64, device=dev)
    _lib.call("nrk_itemcf_recall_offsets", _ptr(q_slot), nq, _ptr(offsets), _ptr(items), _ptr(nbr_cnt),
              _ptr(cand_off), _stream())
    n_cand = int(cand_off[nq].item())
    ws = torch.empty(_lib.lib().nrk_itemcf_recall_workspace_bytes(n_cand), dtype=torch.uint8, device=dev)
    oi = torch.empty((nq, topk), dtype=torch.int32, device=dev)
    osc = torch.empty((nq, topk), dtype=torch.float64, device=dev)
    osrc = torch.empty((nq, topk), dtype=torch.int32, device=dev)
    ocnt = torch.empty(nq, dtype=torch.int32, device=dev)
    _lib.call("nrk_itemcf_recall", _ptr(q_slot), nq, _ptr(offsets), _ptr(items), _ptr(nbr_cols),
              _ptr(nbr_vals), _ptr(nbr_cnt), topn, _ptr(created), n_items, _ptr(hot), hot.numel(),
              _ptr(emb_cols), _ptr(emb_vals), _ptr(emb_cnt), ke, float(loc_beta), float(created_alpha),
              _ptr(cand_off), n_cand, int(topk), _ptr(oi), _ptr(osc), _ptr(osrc), _ptr(ocnt), _ptr(ws),
              ws.numel(), _stream())
    return oi, osc, osrc, ocnt


def din_assemble(rec_rows, rec_scores, user_feat, item_feat, user_hist, hist_len, u0, nu, k_use=30, skip=1,
                 n_ctx=16, ctx_bins=10, score_lo=-1.0, score_hi=1.0, seed=23, out=None, validate=True,
                 ctx_width=None):
    """DIN inputs of the recalled pairs of users [u0, u0 + nu) (nrk_din_assemble).
    Returns dict user [P, Fu], item [P, Fi], hist [P, T, Fi], ctx [P, ctx_width]
    (the first n_ctx columns filled: synthetic score / hash bins),
    mask [P, T] f32, cand [P] (item rows), P = nu * k_use.  ``validate``
    checks every index the kernel gathers (rec_rows, user_hist, hist_len);
    callers that validated their resident tables once pass False."""
    _dev(rec_rows, rec_scores, user_feat, item_feat, user_hist, hist_len)
    n_users, k_in = rec_rows.shape
    _need(rec_rows, torch.int32, name="rec_rows")
    _need(rec_scores, torch.float32, (n_users, k_in), "rec_scores")
    _need(user_feat, torch.int32, name="user_feat")
    _need(item_feat, torch.int32, name="item_feat")
    _need(user_hist, torch.int32, name="user_hist")
    _need(hist_len, torch.int32, (n_users,), "hist_len")
    Fu, Fi, T = user_feat.shape[1], item_feat.shape[1], user_hist.shape[1]
    if user_feat.shape[0] != n_users or user_hist.shape[0] != n_users:
        raise ValueError("user tables must have one row per recalled user")
    if not (0 <= u0 and u0 + nu <= n_users):
        raise ValueError("user range out of bounds")
    if validate and nu:
        n_items = item_feat.shape[0]
        r = rec_rows[u0:u0 + nu]
        if int(r.max()) >= n_items:
            raise ValueError("rec_rows out of [0, n_items)")
        if int(user_hist.min()) < 0 or int(user_hist.max()) >= n_items:
            raise ValueError("user_hist rows out of [0, n_items)")
        if int(hist_len.min()) < 0 or int(hist_len.max()) > T:
            raise ValueError("hist_len out of [0, T]")
    W = n_ctx if ctx_width is None else ctx_width
    if n_ctx and W != n_ctx:
        raise ValueError("ctx_width must equal n_ctx when the assembly fills the context block")
    P = nu * k_use
    dev = rec_rows.device
    if out is None:
        out = {"user": torch.empty((P, Fu), dtype=torch.int32, device=dev),
               "item": torch.empty((P, Fi), dtype=torch.int32, device=dev),
               "hist": torch.empty((P, T, Fi), dtype=torch.int32, device=dev),
               "ctx": torch.empty((P, W), dtype=torch.int32, device=dev),
               "mask": torch.empty((P, T), dtype=torch.float32, device=dev),
               "cand": torch.empty(P, dtype=torch.int32, device=dev)}
    _lib.call("nrk_din_assemble", _ptr(rec_rows), _ptr(rec_scores), n_users, k_in, int(skip), int(k_use),
              _ptr(user_feat), Fu, _ptr(item_feat), item_feat.shape[0], Fi, _ptr(user_hist), _ptr(hist_len), T,
              int(n_ctx), int(ctx_bins), float(score_lo), float(score_hi), int(seed) & 0xFFFFFFFF, int(u0), int(nu),
              _ptr(out["user"]), _ptr(out["item"]), _ptr(out["hist"]), _ptr(out["ctx"]), _ptr(out["mask"]),
              _ptr(out["cand"]), _stream())
    return out


def gather_rows(src, idx):
    """out[b] = src[idx[b]] for a [n_rows, ...] table of 4-byte elements
    (int32 / float32); rows whose index is outside [0, n_rows) are zeros."""
    _dev(src, idx)
    _need(idx, torch.int32, name="idx")
    if src.dtype not in (torch.int32, torch.float32):
        raise ValueError("src must be int32 or float32")
    W = 1
    for d in src.shape[1:]:
        W *= int(d)
    n = idx.numel()
    out = torch.empty((n,) + tuple(src.shape[1:]), dtype=src.dtype, device=idx.device)
    _lib.call("nrk_gather_rows", _ptr(src), src.shape[0], W, _ptr(idx), n, _ptr(out), _stream())
    return out


# ---------------------------------------------------- users-sharded ItemCF --
def itemcf_pairs(offsets, items, ts, created, n_items, slot_base=0, loc_alpha=1.0, loc_alpha_rev=0.7,
                 loc_beta=0.9, time_alpha=0.7, created_alpha=0.8):
    """Pair tuples of a user range (nrk_itemcf_pairs): keys u64 (as int64),
    global slots int32, weights f64, local click counts int64 [n_items]."""
    _dev(offsets, items, ts, created)
    _need(offsets, torch.int64, name="offsets")
    _need(items, torch.int32, (items.numel(),), "items")
    _need(ts, torch.int64, (items.numel(),), "ts")
    _need(created, torch.float64, (n_items,), "created")
    n_users = offsets.numel() - 1
    dev = offsets.device
    pair_off = torch.empty(n_users + 1, dtype=torch.int64, device=dev)
    _lib.call("nrk_itemcf_pair_offsets", _ptr(offsets), n_users, _ptr(pair_off), _stream())
    n = int(pair_off[-1])
    if int(slot_base) < 0 or int(slot_base) + n >= (1 << 31) - (1 << 16):
        raise ValueError("slot_base + pairs must stay below 2^31 (int32 global slots)")
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    slots = torch.empty(n, dtype=torch.int32, device=dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    cnt = torch.zeros(n_items, dtype=torch.int64, device=dev)
    _lib.call("nrk_itemcf_pairs", _ptr(offsets), n_users, _ptr(items), _ptr(ts), _ptr(created), n_items,
              _ptr(pair_off), int(slot_base), float(loc_alpha), float(loc_alpha_rev), float(loc_beta),
              float(time_alpha), float(created_alpha), _ptr(keys), _ptr(slots), _ptr(w), _ptr(cnt), _stream())
    return keys, slots, w, cnt


def itemcf_reduce(keys, slots, w, n_items, item_cnt):
    """The owner's pass (nrk_itemcf_reduce) over tuples in global slot order ->
    ItemCFSim of its items (entries sorted by (i, j))."""
    _dev(keys, slots, w, item_cnt)
    n = keys.numel()
    _need(keys, torch.int64, name="keys")
    _need(slots, torch.int32, (n,), "slots")
    _need(w, torch.float64, (n,), "w")
    _need(item_cnt, torch.int64, (n_items,), "item_cnt")
    dev = item_cnt.device
    cap = max(n, 1)
    oi = torch.empty(cap, dtype=torch.int32, device=dev)
    oj = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    of = torch.empty(cap, dtype=torch.int64, device=dev)
    on = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(_lib.lib().nrk_itemcf_reduce_workspace_bytes(n), dtype=torch.uint8, device=dev)
    _lib.call("nrk_itemcf_reduce", _ptr(keys), _ptr(slots), _ptr(w), n, n_items, _ptr(item_cnt), _ptr(oi),
              _ptr(oj), _ptr(ov), _ptr(of), _ptr(on), _ptr(ws), ws.numel(), _stream())
    m = int(on.item())
    return ItemCFSim(oi[:m], oj[:m], ov[:m], of[:m], item_cnt, n_items)
