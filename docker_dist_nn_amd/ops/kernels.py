"""Tensor-level entry points of the compute kernels.

Every op takes pre-allocated output tensors (the engine owns all step buffers, so a captured HIP
graph replays with fixed pointers) and dispatches on the device of its inputs:

* CUDA/HIP tensors -> the hand-written gfx950 kernels of ``csrc/kernels`` through the native
  extension. There is deliberately NO PyTorch fallback on the GPU: if the extension is missing,
  :func:`docker_dist_nn_amd.utils.native.native` raises.
* CPU tensors -> :mod:`.reference`, a torch implementation with the same numerics contract
  (bf16 operands, fp32 accumulation, bf16/fp32 outputs). It exists so the engine/pipeline/DP
  logic is testable on CPU with the gloo backend, and it is the oracle of the GPU kernel tests.
"""
from __future__ import annotations

import math
import os

import torch

from ..models.mlp import ACT_CODE
from ..utils.native import native
from . import reference as ref
from . import tuning
from .. import switches

KMAJ, MNMAJ = 0, 1


def _parse_stages(spec: str) -> dict:
    """DNN_GEMM_STAGES: "3" (every GEMM) or "fwd=3,dgrad=2,wgrad=4,xent=2"; 0 = kernel
    default."""
    out = {"fwd": 0, "dgrad": 0, "wgrad": 0, "xent": 0}
    spec = spec.strip()
    if not spec:
        return out
    if "=" not in spec:
        return {k: int(spec) for k in out}
    for part in spec.split(","):
        k, v = part.split("=")
        if k.strip() not in out:
            raise ValueError(f"DNN_GEMM_STAGES: unknown GEMM kind {k!r}")
        out[k.strip()] = int(v)
    return out


# LDS pipeline depth (2..4) per GEMM kind; see mma_tile in csrc/kernels/gemm.hip. 8 selects the
# ping-pong half-tile-streamed form of the 256x256 tile (csrc/kernels/gemm_pp.hip).
STAGES = _parse_stages(switches.get("DNN_GEMM_STAGES"))
# A/B of the activation-specialised register-direct epilogue (GemmParams::epi_probe bit 2)
_EPI_GENERIC = 4 if switches.get("DNN_GEMM_EPI_GENERIC") == "1" else 0


def _parse_persist(spec: str) -> dict:
    """DNN_GEMM_PERSIST: "" (tuned table decides), "0"/"1" (every GEMM off/on), or
    "fwd=1,dgrad=0,wgrad=1"; a value > 1 is an explicit workgroup count. None = table."""
    out = {"fwd": None, "dgrad": None, "wgrad": None}
    spec = spec.strip()
    if not spec:
        return out
    if "=" not in spec:
        return {k: int(spec) for k in out}
    for part in spec.split(","):
        k, v = part.split("=")
        if k.strip() not in out:
            raise ValueError(f"DNN_GEMM_PERSIST: unknown GEMM kind {k!r}")
        out[k.strip()] = int(v)
    return out


# Persistent-workgroup GEMM form (csrc/kernels/gemm_persist.hip) per GEMM kind.
PERSIST = _parse_persist(switches.get("DNN_GEMM_PERSIST"))


def _persist(kind: str, entry) -> int:
    """Native `persist` argument: 0 = one tile per workgroup, -1 = one resident round of
    persistent workgroups, > 1 = that many workgroups."""
    v = PERSIST[kind]
    if v is None:
        v = (entry or {}).get("persist", 0)
    return -1 if v == 1 else int(v)


def _blas_requested(kind: str, entry) -> bool:
    """Is the library (hipBLASLt) GEMM requested for this product? DNN_BLAS: "" / "table" = the
    tuned table's ``blas`` flag, "0" = never, "1" = every product the library path supports,
    or per kind ("fwd=1,dgrad=0,wgrad=1")."""
    spec = switches.get("DNN_BLAS").strip()
    if spec in ("", "table"):
        return bool((entry or {}).get("blas", 0))
    if "=" not in spec:
        return spec == "1"
    return dict(kv.split("=") for kv in spec.split(",")).get(kind, "0") == "1"


_BLAS_WARNED = []


def blas_built() -> bool:
    """The library path exists only in the comparison build (``_build --blas``); the product
    build links no vendor GEMM library."""
    return bool(native().blas_available())


def _blas(kind: str, entry) -> bool:
    """Library GEMM for this product: requested (``_blas_requested``) AND built in."""
    if not _blas_requested(kind, entry):
        return False
    if blas_built():
        return True
    if not _BLAS_WARNED:
        _BLAS_WARNED.append(1)
        import warnings

        warnings.warn("DNN_BLAS asks for the hipBLASLt path, which is only in the comparison "
                      "build (python -m docker_dist_nn_amd._build --blas): own kernels run")
    return False


_BLAS_OK: dict = {}


def _blas_ok(a, b, d, trans_a, trans_b, M, N, K, bias, relu, accumulate) -> bool:
    """Does hipBLASLt have an algorithm for this problem signature? (probed once per signature;
    a table entry that asks for the library falls back to the MFMA kernels when it has none)"""
    key = (trans_a, trans_b, M, N, K, a.stride(0), b.stride(0), d.stride(-2),
           d.dtype == torch.float32, bias is not None, relu, accumulate)
    ok = _BLAS_OK.get(key)
    if ok is None:
        ok = _BLAS_OK[key] = bool(native().blas_supported(
            int(trans_a), int(trans_b), M, N, K, a.stride(0), b.stride(0), d.stride(-2),
            int(d.dtype == torch.float32), int(bias is not None), int(relu), int(accumulate)))
    return ok


def blas_gemm(a, b, d, *, trans_a: bool, trans_b: bool, M: int, N: int, K: int, bias=None,
              relu: bool = False, accumulate: bool = False, algo: int = 0):
    """hipBLASLt library GEMM (csrc/runtime/blaslt.hpp), row-major: d[M][N] (+)= op(a).op(b)
    (+ bias, ReLU), a = [M][K] or (trans_a) [K][M], b = [K][N] or (trans_b) [N][K]."""
    if not a.is_cuda:
        raise ValueError("blas_gemm is a GPU path")
    for t, name in ((a, "a"), (b, "b")):
        _rows(t, name, torch.bfloat16)
    if d.dtype not in (torch.bfloat16, torch.float32) or d.stride(-1) != 1:
        raise ValueError("d must be a row-major bf16 or fp32 matrix")
    native().blas_gemm(int(trans_a), int(trans_b), M, N, K, _p(a), a.stride(0), _p(b),
                       b.stride(0), _p(d), d.stride(-2), int(d.dtype == torch.float32),
                       _p(bias), int(relu), int(accumulate), _stream(a), int(algo))


def dact_colsum(x, aux, act, part=None, n_part: int = 1):
    """x = act'(aux) * x in place (bf16), and (optional) part[n_part][cols] = column sums of the
    result over n_part row blocks: the epilogue of a library-GEMM dgrad."""
    rows, cols = x.shape
    if not x.is_cuda:
        x.copy_(ref.act_bwd(x.float(), aux[:rows, :cols].float(), _act(act)).to(x.dtype))
        if part is not None:
            ref.colsum_partial(x, part, n_part)
        return
    native().dact_colsum(_p(x), x.stride(0), _p(aux), aux.stride(0), _act(act), rows, cols,
                         n_part, _p(part), _stream(x))


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _rows(t: torch.Tensor, name: str, dtype: torch.dtype) -> None:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a row-major 2-D tensor, got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


def _act(act) -> int:
    return ACT_CODE[act] if isinstance(act, str) else int(act)


# Residency model for tile choice: LDS/regs admit 2 (128x128), 3 (128x64 / 64x128) or
# 4 (64x64) 4-wave workgroups per CU, and one 8-wave workgroup of the 256-row/-column tiles;
# relative per-CU throughput of the tile shapes.
_TILE_OCC = {(128, 128): 2, (128, 64): 3, (64, 128): 3, (64, 64): 4,
             (256, 256): 1, (256, 128): 1, (128, 256): 1, (256, 64): 1}
_TILE_EFF = {(128, 128): 1.0, (128, 64): 0.82, (64, 128): 0.82, (64, 64): 0.62}
BIG_TILES = [(256, 256), (256, 128), (128, 256), (256, 64)]
NUM_CU = 256


def pick_tiles(M: int, N: int, splits: int = 1) -> tuple[int, int]:
    """Tile for a [M][N] output (fwd / dgrad, M = batch rows).

    The 8-wave 256-row tiles stage half the LDS bytes per FLOP of the 128x128 tile and win
    whenever they still give >= 2 workgroups per CU (bench/stage_sweep.py on MI355X): 256x256
    for outputs >= 1024 wide, 256x64 for 128..1023. Otherwise: the 4-wave tile minimising
    modelled time = rounds of resident tiles x per-tile cost."""
    if splits == 1 and M % 256 == 0:
        if N % 256 == 0 and N >= 1024 and (M // 256) * (N // 256) >= 2 * NUM_CU:
            return 256, 256
        if N % 64 == 0 and N >= 128 and (M // 256) * (N // 64) >= 2 * NUM_CU:
            return 256, 64
    best, best_t = None, math.inf
    for (bm, bn) in _TILE_EFF:  # calibrated tiles only
        if M % bm or N % bn:
            continue
        tiles = (M // bm) * (N // bn) * splits
        # tiles resident on one CU share its matrix pipe: time ~ tiles per CU x tile cost
        t = math.ceil(tiles / NUM_CU) * bm * bn / _TILE_EFF[(bm, bn)]
        if t < best_t - 1e-9:
            best, best_t = (bm, bn), t
    if best is None:
        raise ValueError(f"no tile divides M={M}, N={N} (pad to multiples of 64)")
    return best


def pick_splits(M: int, N: int, K_total: int, max_splits: int = 48) -> int:
    """Split-K factor for the batch-contraction (wgrad) GEMM.

    Splits may be uneven (k-ranges differ by at most one 64-step), so any S works. Resident
    workgroups share a CU, so time ~ ceil(tiles*S / CUs) / S tile-times (wave quantisation);
    each extra split adds an fp32 slab of M*N to write and re-read. E.g. 52 tiles: S=8 puts 2
    workgroups on 160 CUs and 1 on 96 (81% busy); S=14 gives 2-3 per CU (95%)."""
    return wgrad_config(M, N, K_total, max_splits)[2]


def wgrad_config(M: int, N: int, K_total: int, max_splits: int = 48) -> tuple[int, int, int]:
    """Joint (bm, bn, splits) choice for the batch-contraction GEMM (see pick_splits): the
    tuned table's measured optimum when it has the shape, else the model below."""
    t = tuning.lookup("wgrad", M, N, K_total)
    if _blas("wgrad", t):  # the library GEMM contracts all rows in one fp32 output
        return (t["tile"][0], t["tile"][1], 1) if t else (*pick_tiles(M, N), 1)
    if t is not None:
        return t["tile"][0], t["tile"][1], t["splits"]
    ksteps = K_total // 64
    slab_cost = 2.0 * M * N * 4 / 5.0e12 * 0.6e15 / NUM_CU  # slab bytes in tile-FLOP units
    best, best_c = None, math.inf
    for (bm, bn), eff in _TILE_EFF.items():
        if M % bm or N % bn:
            continue
        tiles = (M // bm) * (N // bn)
        tile_flops = 2.0 * bm * bn * K_total / eff
        for s in range(1, min(max_splits, ksteps) + 1):
            c = math.ceil(tiles * s / NUM_CU) / s * tile_flops + (s > 1) * s * slab_cost
            if c < best_c * 0.995:
                best, best_c = (bm, bn, s), c
    if best is None:
        raise ValueError(f"no tile divides [{M}][{N}]")
    return best


def gemm(a, b, c, *, layout_a: int, layout_b: int, M: int, N: int, K: int, bias=None, aux=None,
         act=0, accumulate: bool = False, splits: int = 1, tiles: tuple[int, int] | None = None,
         colsum=None, k_total: int = 0, stages: int = 0, group_m: int = 0, persist: int = 0,
         mask_out=None, mask_in=None, ct=None, upd=None, timeline=None, epi_probe: int = 0):
    """C (+)= epilogue(A.B). See csrc/kernels/gemm.hpp for the layout/epilogue contract.
    ``epi_probe`` (diagnosis only, results WRONG): GemmParams::epi_probe.

    ``timeline`` (int64 GPU tensor, >= 4 per workgroup; one-tile kernels): per-workgroup phase
    timestamps for bench/probes/gemm_timeline.py (GemmParams::timeline).

    ``persist`` != 0 runs the persistent-workgroup form with the register-direct epilogue
    (csrc/kernels/gemm_persist.hip): -1 = one resident round, > 0 = workgroup count.
    ``mask_out`` / ``mask_in`` (uint8 [M][>= N/8], act = relu, GPU only): the forward writes the
    1-bit ReLU mask of its stored output; a dgrad reads it instead of ``aux``.

    ``k_total`` > 0 selects uneven split-K over the full contraction length (K is ignored).
    ``colsum`` (bf16 output only): fp32 [M/bm][>=N] receives per-row-tile column sums of the
    stored output; requires explicit ``tiles`` so the caller knows the partial count."""
    if k_total:
        K = k_total
    act = _act(act)
    out_f32 = c.dtype == torch.float32
    if colsum is not None:
        if tiles is None or out_f32:
            raise ValueError("colsum needs explicit tiles and a bf16 output")
        if colsum.dtype != torch.float32 or colsum.dim() != 2 or colsum.stride(1) != 1 or \
                colsum.shape[0] < -(-M // tiles[0]) or colsum.shape[1] < N:
            raise ValueError(f"colsum must be fp32 [{-(-M // tiles[0])}][>={N}] row-major")
    if (mask_out is not None or mask_in is not None) and not a.is_cuda:
        raise ValueError("relu bit masks are a GPU-path format (CPU uses aux)")
    frag = isinstance(mask_out, FragMask) or isinstance(mask_in, FragMask)
    for m in (mask_out, mask_in):
        if isinstance(m, FragMask):
            if tiles is None or tuple(tiles) != m.tiles or stages not in DIRECT_STAGES or \
                    m.m < M or m.n < N or m.buf.numel() < FragMask.nbytes(M, N, m.tiles):
                raise ValueError(f"fragment mask of tile {m.tiles} [{m.m}][{m.n}] used by a "
                                 f"{tiles} GEMM (stage code {stages}) of [{M}][{N}]")
        elif m is not None and frag:
            raise ValueError("mask_out and mask_in must share one layout")
    for m in () if frag else (mask_out, mask_in):  # row-block-major bytes (relu_mask_bits)
        if m is not None and (m.dtype != torch.uint8 or m.dim() != 2 or not m.is_contiguous() or
                              M % 16 or m.shape[0] < M or m.shape[1] < -(-N // 8)):
            raise ValueError(f"relu mask must be a contiguous uint8 [{M}][>={-(-N // 8)}] "
                             "tensor and M a multiple of 16")
    if ct is not None and (ct.dtype != torch.bfloat16 or ct.dim() != 2 or ct.stride(1) != 1 or
                           ct.shape[0] < N or ct.shape[1] < M or (out_f32 and upd is None)):
        raise ValueError(f"ct must be a bf16 [>={N}][>={M}] row-major transposed output")
    if upd is not None:
        # fused SGD epilogue (f32 output of one split): the gradient updates the weights in place
        # -- upd = dict(master=fp32 [M][N] view (row stride = C's), mom=None | same shape,
        # shadow=None | bf16 same shape, lr_dev=fp32 [1], momentum, weight_decay); ct = W^T
        if not out_f32 or splits != 1 or accumulate or bias is not None:
            raise ValueError("fused update: f32 output, one split, no accumulation / bias")
        for k in ("master", "mom", "shadow"):
            t = upd.get(k)
            if t is not None and (t.dim() != 2 or t.stride(1) != 1 or t.shape[0] < M or
                                  t.shape[1] < N or t.stride(0) != (c if c.dim() == 2
                                                                    else c[0]).stride(0)):
                raise ValueError(f"fused update: {k} must be [M][N] with C's row stride")
    if stages in DIRECT_STAGES and (ct is not None or upd is not None):
        stages = 6  # the register-direct epilogue has neither: RP loop, staged epilogue
    if not a.is_cuda:
        ref.gemm(a, b, c, layout_a=layout_a, layout_b=layout_b, M=M, N=N, K=K, bias=bias,
                 aux=aux, act=act, accumulate=accumulate, splits=splits, colsum=colsum,
                 colsum_rows=tiles[0] if tiles else 0, k_total=k_total)
        if upd is not None:
            g = (c if c.dim() == 2 else c[0])[:M, :N]
            mom = upd.get("mom")
            sh = upd.get("shadow")
            ref.sgd_update(upd["master"][:M, :N], g, mom[:M, :N] if mom is not None else None,
                           sh[:M, :N] if sh is not None else None, float(upd["lr_dev"][0]),
                           upd.get("momentum", 0.0), upd.get("weight_decay", 0.0))
            if ct is not None:
                ct[:N, :M] = upd["master"][:M, :N].t().to(torch.bfloat16)
            return c
        if ct is not None:
            ct[:N, :M] = c[:M, :N].t()
        return c
    _rows(a, "A", torch.bfloat16)
    _rows(b, "B", torch.bfloat16)
    if splits > 1:
        if c.dim() != 3 or c.shape[0] < splits:
            raise ValueError("split-K output must be [splits][M][N] fp32")
        c_rows, split_stride = c[0], c.stride(0)
    else:
        c_rows, split_stride = (c if c.dim() == 2 else c[0]), 0
    _rows(c_rows, "C", torch.float32 if out_f32 else torch.bfloat16)
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() < N):
        raise ValueError("bias must be fp32 with >= N entries")
    if aux is not None:
        _rows(aux, "aux", torch.bfloat16)
    # shape checks against the storage the kernel will touch
    ka = k_total or K * splits
    need_a = (M, ka) if layout_a == KMAJ else (ka, M)
    need_b = (N, ka) if layout_b == KMAJ else (ka, N)
    if a.shape[0] < need_a[0] or a.shape[1] < need_a[1]:
        raise ValueError(f"A storage {tuple(a.shape)} too small for {need_a}")
    if b.shape[0] < need_b[0] or b.shape[1] < need_b[1]:
        raise ValueError(f"B storage {tuple(b.shape)} too small for {need_b}")
    if c_rows.shape[0] < M or c_rows.shape[1] < N:
        raise ValueError(f"C storage {tuple(c_rows.shape)} too small for {(M, N)}")
    if aux is not None and (aux.shape[0] < M or aux.shape[1] < N):
        raise ValueError("aux storage too small")
    bm, bn = tiles or pick_tiles(M, N, splits)
    # M or N not a multiple of the tile runs as partial edge tiles in the same launch:
    # out-of-range operand rows/columns are clamped on load and never stored (gemm.hip)
    native().gemm_bf16(_p(a), a.stride(0), _p(b), b.stride(0), _p(c_rows), c_rows.stride(0),
                       split_stride, _p(bias), _p(aux), aux.stride(0) if aux is not None else 0,
                       M, N, K, act, int(accumulate), layout_a, layout_b, int(out_f32), bm, bn,
                       splits, _stream(a), _p(colsum),
                       colsum.stride(0) if colsum is not None else 0, k_total=int(k_total),
                       stages=int(stages), group_m=int(group_m), persist=int(persist),
                       mask_out=_p(mask_out.buf if frag and mask_out is not None else mask_out),
                       mask_in=_p(mask_in.buf if frag and mask_in is not None else mask_in),
                       ld_mask=-1 if frag else
                       (mask_out if mask_out is not None else mask_in).stride(0)
                       if (mask_out is not None or mask_in is not None) else 0,
                       ct=_p(ct), ld_ct=ct.stride(0) if ct is not None else 0,
                       **({} if upd is None else dict(
                           upd_master=_p(upd["master"]), upd_mom=_p(upd.get("mom")),
                           upd_shadow=_p(upd.get("shadow")), upd_lr=_p(upd["lr_dev"]),
                           upd_mu=float(upd.get("momentum", 0.0)),
                           upd_wd=float(upd.get("weight_decay", 0.0)))),
                       timeline=_p(timeline), epi_probe=int(epi_probe) | _EPI_GENERIC)
    return c


# ---- the three GEMMs of a Linear layer -----------------------------------------------------

GEMV_MAX_ROWS = 8


def gemv(x, w, bias, y, act="relu"):
    """Serving-size layer (1..8 rows): y[m][n] = act(x[m] . w[n] + bias[n]), one wave per
    output neuron (csrc/kernels/gemv.hip). y bf16 or fp32."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:
        return ref.gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=bias,
                        act=_act(act))
    if M > GEMV_MAX_ROWS or K % 8:
        raise ValueError(f"gemv takes <= {GEMV_MAX_ROWS} rows and K % 8 == 0")
    _rows(x, "x", torch.bfloat16)
    _rows(w, "w", torch.bfloat16)
    if w.shape[1] < K or y.shape[0] < M or y.shape[1] < N or y.stride(1) != 1:
        raise ValueError("gemv operand shapes do not match")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() < N):
        raise ValueError("bias must be fp32 with >= N entries")
    native().gemv_bf16(_p(x), x.stride(0), _p(w), w.stride(0), _p(bias), _p(y), y.stride(0),
                       M, N, K, _act(act), int(y.dtype == torch.float32), _stream(x))
    return y


# wave grid (WM, WN) of the register-direct tiles that take fragment-order masks (NB >= 4 bytes
# per lane; gemm_rp.hip pick_rp)
FRAG_WAVES = {(256, 256): (4, 2), (256, 128): (4, 2), (128, 128): (2, 2), (128, 64): (2, 2)}
DIRECT_STAGES = (9, 11)


class FragMask:
    """1-bit ReLU mask in FRAGMENT order (GemmParams::ld_mask < 0, gemm_tile.hpp
    frag_mask_offset): the bits a lane of the register-direct epilogue stores or reads are
    contiguous, so one 4/8/16-byte access per lane moves them, instead of the row-block-major
    layout's one-byte accesses (the reason DNN_RELU_MASK=1 measured slower than reading the
    activation). Tied to one tile shape: the forward that writes it and the dgrad that reads it
    must both run ``tiles`` with a register-direct stage code. Tiles are row-major in the
    buffer, so the rows of a micro-batch starting on a tile boundary are one byte range
    (``mask[r]`` with r a slice of rows)."""

    def __init__(self, buf: torch.Tensor, tiles: tuple[int, int], m: int, n: int):
        self.buf, self.tiles, self.m, self.n = buf, tuple(tiles), m, n

    @staticmethod
    def nbytes(M: int, N: int, tiles) -> int:
        bm, bn = tiles
        return -(-M // bm) * -(-N // bn) * bm * bn // 8

    @classmethod
    def alloc(cls, M: int, N: int, tiles, device) -> "FragMask":
        if tuple(tiles) not in FRAG_WAVES:
            raise ValueError(f"no fragment-order mask for tile {tuple(tiles)}")
        return cls(torch.zeros(cls.nbytes(M, N, tiles), dtype=torch.uint8, device=device),
                   tiles, M, N)

    def __getitem__(self, r: slice) -> "FragMask":
        bm, bn = self.tiles
        start, stop, step = r.indices(self.m)
        if step != 1 or start % bm:
            raise ValueError(f"fragment mask rows must start on a {bm}-row tile boundary")
        per_row_tile = -(-self.n // bn) * bm * bn // 8
        return FragMask(self.buf[start // bm * per_row_tile:], self.tiles, stop - start, self.n)

    def bits(self) -> torch.Tensor:
        """Unpack into bool [m][n] (tests)."""
        bm, bn = self.tiles
        wm_n, wn_n = FRAG_WAVES[self.tiles]
        fm, sn = bm // wm_n // 16, bn // wn_n
        fn = sn // 16
        tm_n, tn_n = -(-self.m // bm), -(-self.n // bn)
        dev = self.buf.device
        raw = self.buf[:tm_n * tn_n * bm * bn // 8].view(tm_n, tn_n, wm_n, wn_n, 64, fn // 2, fm)
        ar = lambda k: torch.arange(k, device=dev)  # noqa: E731
        tm, tn, wm, wn, lane, jj, i, e = torch.meshgrid(
            ar(tm_n), ar(tn_n), ar(wm_n), ar(wn_n), ar(64), ar(fn // 2), ar(fm), ar(8),
            indexing="ij")
        row = tm * bm + wm * 16 * fm + (lane & 15) + 16 * i
        col = tn * bn + wn * sn + 16 * ((lane >> 4) & 1) + 8 * (lane >> 5) + 32 * jj + e
        bit = (raw.unsqueeze(-1).to(torch.int32) >> ar(8).to(torch.int32)) & 1
        out = torch.zeros(tm_n * bm, tn_n * bn, dtype=torch.bool, device=dev)
        out[row.reshape(-1), col.reshape(-1)] = bit.reshape(-1).bool()
        return out[:self.m, :self.n]


def frag_mask_tiles(M: int, N: int, K: int, N_next: int) -> tuple[int, int] | None:
    """Tile of a fragment-order mask between the forward [M][N] (contraction K) of a ReLU layer
    and the dgrad that produces its dZ from the next layer's [M][N_next] gradient, or None when
    those two GEMMs do not both run one register-direct tile shape (linear_fwd / linear_dgrad
    pick their tiles and stage codes from the tuned table)."""
    tf = tuning.lookup("fwd", M, N, K)
    tiles = tuple(tf["tile"]) if tf else pick_tiles(M, N)
    td = tuning.lookup("dgrad", M, N, N_next)
    sf = STAGES["fwd"] or (tf or {}).get("stages", 0)
    sd = STAGES["dgrad"] or (td or {}).get("stages", 0)
    if M <= GEMV_MAX_ROWS or tiles != dgrad_tiles(M, N, N_next) or tiles not in FRAG_WAVES or \
            sf not in DIRECT_STAGES or sd not in DIRECT_STAGES or M % tiles[0] or \
            _blas("fwd", tf) or _blas("dgrad", td):
        return None
    return tiles


def relu_mask_bits(mask: torch.Tensor, M: int, N: int) -> torch.Tensor:
    """Unpack a GEMM-written ReLU mask (uint8 [M][ld], row-block-major: the byte of row r,
    8-column chunk c is at flat index ((r // 16) * ld + c) * 16 + r % 16) into bool [M][N]."""
    ld = mask.shape[1]
    blocks = mask.reshape(-1)[:M * ld].view(M // 16, ld, 16).transpose(1, 2).reshape(M, ld)
    bits = (blocks[:, :(N + 7) // 8].to(torch.int32).unsqueeze(-1) >>
            torch.arange(8, device=mask.device, dtype=torch.int32)) & 1
    return bits.reshape(M, -1)[:, :N].bool()


def linear_fwd(x, w, bias, y, act="relu", mask=None, yt=None):
    """y[M][Np] = act(x[M][Kp] . w[Np][Kp]^T + bias). y bf16 (activation) or fp32 (logits).
    M <= 8 rows (serving) runs the GEMV kernel; otherwise the MFMA GEMM. ``mask`` (GPU, relu):
    also write the 1-bit mask of y for the next dgrad. ``yt`` (bf16 [Np][>=M], may be a column
    slice): also write y transposed (the next layer's weight gradient reads it K-major)."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:  # CPU reference: any row count
        return gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=bias, act=act,
                    ct=yt)
    if M <= GEMV_MAX_ROWS:
        return gemv(x, w, bias, y, act)
    t = tuning.lookup("fwd", M, N, K)
    if mask is None and act in ("relu", "linear", 0, 1) and _blas("fwd", t) and \
            _blas_ok(x, w, y, False, True, M, N, K, bias, _act(act) == 1, False):
        return blas_gemm(x, w, y, trans_a=False, trans_b=True, M=M, N=N, K=K, bias=bias,
                         relu=_act(act) == 1, algo=(t or {}).get("blas_algo", 0))
    tiles = tuple(t["tile"]) if t else pick_tiles(M, N)
    return gemm(x, w, y, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=bias, act=act,
                tiles=tiles, stages=STAGES["fwd"] or (t or {}).get("stages", 0),
                persist=0 if (mask is not None or yt is not None) else _persist("fwd", t),
                mask_out=mask, ct=yt)


def xent_tiles(M: int, N: int) -> tuple[int, int]:
    """Tile of the fused linear+softmax-CE GEMM: the whole padded row in one tile (bn == N)."""
    if N not in (64, 128):
        raise ValueError(f"fused cross-entropy supports 64 or 128 padded classes, got {N}")
    bm = 128 if M % 128 == 0 and (M // 128) * 1 >= NUM_CU // 2 else 64
    if M % bm:
        raise ValueError("rows must be a multiple of 64")
    return bm, N


def linear_fwd_xent(x, w, bias, dz, labels, n_cls, scale, loss_part=None, correct=None,
                    colsum=None):
    """Last layer + softmax cross-entropy in ONE kernel: dz[M][Np] = (softmax(x.w^T + b) -
    onehot) * scale; loss_part[M/bm] per-tile loss sums; correct[M/bm] per-tile #argmax==label;
    colsum[M/bm][Np] = per-tile column sums of dz (the bias-gradient partials)."""
    M, K = x.shape
    N = w.shape[0]
    bm, bn = xent_tiles(M, N)
    if labels.dtype != torch.int32 or labels.numel() < M:
        raise ValueError("labels must be int32 with one entry per row")
    if loss_part is not None and loss_part.numel() < M // bm:
        raise ValueError(f"loss_part needs {M // bm} entries")
    if correct is not None and (correct.dtype != torch.int32 or correct.numel() < M // bm):
        raise ValueError(f"correct needs {M // bm} int32 entries")
    if not x.is_cuda:
        logits = torch.empty(M, N, dtype=torch.float32)
        ref.gemm(x, w, logits, layout_a=KMAJ, layout_b=KMAJ, M=M, N=N, K=K, bias=bias)
        ref.softmax_xent(logits, labels, dz, n_cls, scale, loss_part, correct, bm, colsum)
        return dz
    _rows(x, "x", torch.bfloat16)
    _rows(w, "w", torch.bfloat16)
    _rows(dz, "dz", torch.bfloat16)
    if colsum is not None and (colsum.dtype != torch.float32 or colsum.shape[0] < M // bm or
                               colsum.shape[1] < N or colsum.stride(1) != 1):
        raise ValueError(f"colsum must be fp32 [{M // bm}][>={N}]")
    if bias is None or bias.dtype != torch.float32 or bias.numel() < N:
        raise ValueError("fused cross-entropy needs an fp32 bias")
    native().gemm_bf16(_p(x), x.stride(0), _p(w), w.stride(0), _p(dz), dz.stride(0), 0,
                       _p(bias), 0, 0, M, N, K, 0, 0, KMAJ, KMAJ, 0, bm, bn, 1, _stream(x),
                       _p(colsum), colsum.stride(0) if colsum is not None else 0, _p(labels),
                       int(n_cls), float(scale), _p(loss_part), _p(correct),
                       stages=STAGES["xent"])
    return dz


def dgrad_tiles(M: int, K: int, N: int = 0) -> tuple[int, int]:
    """Tile shape used by linear_dgrad for an [M][K] output from an [M][N] gradient (fixes
    the colsum partial count)."""
    t = tuning.lookup("dgrad", M, K, N) if N else None
    return tuple(t["tile"]) if t else pick_tiles(M, K, 1)


def transpose_bf16(src, dst):
    """dst[c][r] = src[r][c] (bf16, both dims multiples of 64)."""
    rows, cols = src.shape
    if dst.shape[0] < cols or dst.shape[1] < rows:
        raise ValueError(f"transpose_bf16: dst {tuple(dst.shape)} too small for {(cols, rows)}")
    if not src.is_cuda:
        dst[:cols, :rows] = src.t()
        return dst
    _rows(src, "src", torch.bfloat16)
    _rows(dst, "dst", torch.bfloat16)
    native().transpose_bf16(_p(src), src.stride(0), rows, cols, _p(dst), dst.stride(0),
                            _stream(src))
    return dst


def transpose_multi(pairs):
    """transpose_bf16 for every (src, dst) pair, one launch on the GPU (<= 16 pairs)."""
    pairs = list(pairs)
    if not pairs:
        return
    if not pairs[0][0].is_cuda:
        for src, dst in pairs:
            transpose_bf16(src, dst)
        return
    jobs = []
    for src, dst in pairs:
        rows, cols = src.shape
        _rows(src, "src", torch.bfloat16)
        _rows(dst, "dst", torch.bfloat16)
        if dst.shape[0] < cols or dst.shape[1] < rows:
            raise ValueError("transpose_multi: dst too small")
        jobs.append((_p(src), src.stride(0), rows, cols, _p(dst), dst.stride(0)))
    for k in range(0, len(jobs), 16):
        native().transpose_multi(jobs[k:k + 16], _stream(pairs[0][0]))


FP8_MAX = 448.0  # OCP e4m3 (gfx950's fp8; not the fnuz variant of MI300)


def quant_rows_fp8(x, q, scale):
    """Pipeline-boundary compression: q[r] = e4m3(x[r] / scale[r]), scale[r] = amax(x[r])/448.
    x bf16 [rows][cols], q uint8 [rows][>=cols], scale fp32 [rows]."""
    rows, cols = x.shape
    if q.dtype != torch.uint8 or q.shape[0] < rows or q.shape[1] < cols or scale.numel() < rows:
        raise ValueError("quant_rows_fp8: q must be uint8 [rows][>=cols], scale fp32 [>=rows]")
    if not x.is_cuda:
        xf = x.float()
        amax = xf.abs().amax(1)
        inv = torch.where(amax > 0, FP8_MAX / amax, torch.zeros_like(amax))
        q[:rows, :cols] = (xf * inv[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
        scale[:rows] = amax / FP8_MAX
        return
    _rows(x, "x", torch.bfloat16)
    native().quant_rows_fp8(_p(x), x.stride(0), rows, cols, _p(q), q.stride(0), _p(scale),
                            _stream(x))


def dequant_rows_fp8(q, scale, x):
    """Inverse of quant_rows_fp8 into bf16 x [rows][cols]."""
    rows, cols = x.shape
    if not x.is_cuda:
        v = q[:rows, :cols].view(torch.float8_e4m3fn).float() * scale[:rows, None]
        x.copy_(v.to(torch.bfloat16))
        return
    _rows(x, "x", torch.bfloat16)
    native().dequant_rows_fp8(_p(q), q.stride(0), _p(scale), rows, cols, _p(x), x.stride(0),
                              _stream(x))


def linear_dgrad(dz, w, dx, y_prev=None, act_prev="linear", colsum=None, mask_prev=None,
                 wt=None, dxt=None):
    """dx[M][Kp] = (dz[M][Np] . w[Np][Kp]) * act_prev'(y_prev) (mask fused in the epilogue).
    ``colsum`` [M/bm][Kp] receives the bias-gradient partials of the PREVIOUS layer (column
    sums of dx), fused in the same epilogue. ``wt`` = w^T [Kp][Np] (the transposed weight
    shadow): the GEMM then reads both operands contraction-contiguous -- the forward's main
    loop, 1.2-1.25x faster than transposing w per tile (bench/layout_ab.py) -- with the same
    MFMA k order, so the result is bitwise identical."""
    M, N = dz.shape
    K = w.shape[1]
    if mask_prev is not None:  # relu derivative from the forward's 1-bit mask
        y_prev, act_prev = None, "relu"
    elif y_prev is None:
        act_prev = "linear"
    t = tuning.lookup("dgrad", M, K, N)
    if mask_prev is None and dz.is_cuda and _blas("dgrad", t) and \
            _blas_ok(dz, w, dx, False, False, M, K, N, None, False, False):
        blas_gemm(dz, w, dx, trans_a=False, trans_b=False, M=M, N=K, K=N,
                  algo=(t or {}).get("blas_algo", 0))
        n_part = -(-M // dgrad_tiles(M, K, N)[0])
        if y_prev is not None and _act(act_prev) != 0:
            dact_colsum(dx, y_prev, act_prev, colsum, n_part)
        elif colsum is not None:
            colsum_partial(dx, colsum, n_part)
        return dx
    if wt is not None and dz.is_cuda:
        return gemm(dz, wt, dx, layout_a=KMAJ, layout_b=KMAJ, M=M, N=K, K=N, aux=y_prev,
                    act=act_prev, tiles=dgrad_tiles(M, K, N), colsum=colsum,
                    stages=STAGES["dgrad"] or (t or {}).get("stages", 0),
                    persist=0 if (dxt is not None or mask_prev is not None)
                    else _persist("dgrad", t), mask_in=mask_prev, ct=dxt)
    return gemm(dz, w, dx, layout_a=KMAJ, layout_b=MNMAJ, M=M, N=K, K=N, aux=y_prev,
                act=act_prev, tiles=dgrad_tiles(M, K, N), colsum=colsum,
                stages=STAGES["dgrad"] or (t or {}).get("stages", 0),
                persist=0 if (mask_prev is not None or dxt is not None)
                else _persist("dgrad", t), mask_in=mask_prev, ct=dxt)


def linear_wgrad(dz, x, slabs, splits=1, accumulate=False, dzt=None, xt=None, upd=None,
                 wt=None):
    """slabs[s][Np][Kp] (+)= dz[rows_s]^T . x[rows_s] over the batch rows of split s (fp32).
    ``dzt`` / ``xt`` (bf16 [Np][R] / [Kp][R], written transposed by the producing GEMMs'
    epilogues): the contraction runs K-major on both operands (the forward's main loop,
    bench/layout_ab.py: 1.2x on 8192x8192 weights); same k order, same result bits.
    ``upd`` (one split): the epilogue applies the SGD step to the layer's weights instead of
    storing the gradient (ops.gemm), and writes the new bf16 weights transposed into ``wt``."""
    R, N = dz.shape
    K = x.shape[1]
    if upd is not None and (splits != 1 or accumulate):
        raise ValueError("the fused weight update needs one split and no accumulation")
    if dzt is not None and xt is not None and dz.is_cuda:
        bm, bn, s = wgrad_config(N, K, R)
        tiles = (bm, bn) if s == splits else pick_tiles(N, K, splits)
        t = tuning.lookup("wgrad", N, K, R) if s == splits else None
        return gemm(dzt, xt, slabs, layout_a=KMAJ, layout_b=KMAJ, M=N, N=K, K=R, k_total=R,
                    accumulate=accumulate, splits=splits, tiles=tiles,
                    stages=STAGES["wgrad"] or (t or {}).get("stages", 0),
                    persist=0 if upd is not None else _persist("wgrad", t), upd=upd, ct=wt)
    if R % 64 or splits > R // 64:
        raise ValueError("rows must be a multiple of 64 with at least 64 rows per split")
    bm, bn, s = wgrad_config(N, K, R)
    tiles = (bm, bn) if s == splits else pick_tiles(N, K, splits)
    t = tuning.lookup("wgrad", N, K, R) if s == splits else None
    if upd is None and splits == 1 and dz.is_cuda and \
            _blas("wgrad", tuning.lookup("wgrad", N, K, R)) and \
            _blas_ok(dz, x, slabs[0], True, False, N, K, R, None, False, accumulate):
        return blas_gemm(dz, x, slabs[0], trans_a=True, trans_b=False, M=N, N=K, K=R,
                         accumulate=accumulate,
                         algo=(tuning.lookup("wgrad", N, K, R) or {}).get("blas_algo", 0))
    return gemm(dz, x, slabs, layout_a=MNMAJ, layout_b=MNMAJ, M=N, N=K, K=R, k_total=R,
                accumulate=accumulate, splits=splits, tiles=tiles,
                stages=STAGES["wgrad"] or (t or {}).get("stages", 0),
                persist=0 if upd is not None else _persist("wgrad", t), upd=upd, ct=wt)


def linear_wgrad_group(items) -> list:
    """Several linear_wgrad calls -- items of (dz, x, slabs, splits, accumulate) -- with the
    items that share a one-tile 4-wave configuration (same tile, 2 stages, not persistent, not
    the library path) and that alone fill less than one round of the chip run as ONE grouped
    launch per configuration (gemm.hip gemm_group_kernel): small latency-bound weight gradients
    then run concurrently (batch-64 recipe step 0.034 -> 0.029 ms); big ones keep their own
    launch (grouping the mlp8 1024x1024 wgrads measured +0.4 %). Returns the indices it did NOT
    launch (the caller runs linear_wgrad for those)."""
    if not items or not items[0][0].is_cuda:
        return list(range(len(items)))
    groups, rest = {}, []
    for idx, (dz, x, slabs, splits, acc) in enumerate(items):
        R, N = dz.shape
        K = x.shape[1]
        bm, bn, s = wgrad_config(N, K, R)
        t = tuning.lookup("wgrad", N, K, R)
        stages = STAGES["wgrad"] or (t or {}).get("stages", 0) or 2
        small = -(-N // bm) * -(-K // bn) * splits < int(
            switches.get("DNN_WGRAD_GROUP_MAX_WG"))  # under one round of the chip
        if (R % 64 or splits > R // 64 or s != splits or _persist("wgrad", t) or
                _blas("wgrad", t) or stages != 2 or not small or
                (bm, bn) not in ((64, 64), (64, 128), (128, 64), (128, 128))):
            rest.append(idx)
            continue
        groups.setdefault((bm, bn), []).append(idx)
    for (bm, bn), idxs in groups.items():
        if len(idxs) < 2:
            rest += idxs
            continue
        for c0 in range(0, len(idxs), 8):
            probs = []
            for idx in idxs[c0:c0 + 8]:
                dz, x, slabs, splits, acc = items[idx]
                R, N = dz.shape
                K = x.shape[1]
                _rows(dz, "dz", torch.bfloat16)
                _rows(x, "x", torch.bfloat16)
                if slabs.dim() != 3 or slabs.shape[0] < splits or slabs.dtype != torch.float32 \
                        or slabs.shape[1] < N or slabs.shape[2] < K or slabs[0].stride(1) != 1:
                    raise ValueError("split-K output must be [splits][N][K] fp32")
                probs.append((_p(dz), dz.stride(0), _p(x), x.stride(0), _p(slabs),
                              slabs.stride(1), slabs.stride(0), N, K, R, R, int(acc), splits))
            native().gemm_bf16_group(probs, MNMAJ, MNMAJ, 1, bm, bn, 2, _stream(items[0][0]))
    return sorted(rest)


STREAMK_WG = 2 * NUM_CU  # stream-K workgroups: two resident per CU, every CU equally loaded


def streamk_tiles(N: int, K: int) -> tuple[int, int]:
    """Output tile of the [N][K] weight gradient: largest tile that divides it."""
    for t in ((128, 128), (128, 64), (64, 128), (64, 64)):
        if N % t[0] == 0 and K % t[1] == 0:
            return t
    raise ValueError(f"weight shape [{N}][{K}] is not 64-aligned")


def streamk_partial_elems(N: int, K: int, nwg: int = STREAMK_WG) -> int:
    bm, bn = streamk_tiles(N, K)
    tiles = (N // bm) * (K // bn)
    return max(nwg, tiles) * 2 * bm * bn


def linear_wgrad_streamk(dz, x, grad_w, part, accumulate=False, nwg: int = STREAMK_WG):
    """grad_w[Np][Kp] (+)= dz^T . x over ALL rows, stream-K balanced; ``part`` is fp32 scratch
    of streamk_partial_elems(Np, Kp) elements."""
    R, N = dz.shape
    K = x.shape[1]
    if not dz.is_cuda:
        g = dz.float().t() @ x.float()
        if accumulate:
            grad_w += g
        else:
            grad_w.copy_(g)
        return grad_w
    _rows(dz, "dz", torch.bfloat16)
    _rows(x, "x", torch.bfloat16)
    _rows(grad_w, "grad_w", torch.float32)
    if x.shape[0] != R or grad_w.shape[0] < N or grad_w.shape[1] < K or R % 64:
        raise ValueError("wgrad shapes do not match")
    if part.dtype != torch.float32 or part.numel() < streamk_partial_elems(N, K, nwg):
        raise ValueError("stream-K partial buffer too small")
    bm, bn = streamk_tiles(N, K)
    native().gemm_bf16_streamk(_p(dz), dz.stride(0), _p(x), x.stride(0), _p(grad_w),
                               grad_w.stride(0), N, K, R, int(accumulate), MNMAJ, MNMAJ, bm, bn,
                               nwg, _p(part), _stream(dz))
    return grad_w


# ---- loss / reductions / optimizers ----------------------------------------------------------

XENT_ROWS_PER_BLOCK = 64  # csrc/kernels/elementwise.hip XENT_ROWS_PER_BLOCK


def xent_blocks(rows: int) -> int:
    """Number of per-block loss partials softmax_xent writes for ``rows`` rows."""
    return -(-rows // XENT_ROWS_PER_BLOCK)


def softmax_xent(logits, labels, dz, n_cls, scale, loss_part=None, correct=None, colsum=None):
    """dz = (softmax - onehot) * scale; per 64-row block: loss partial sum -> loss_part,
    #argmax==label -> correct (int32), and (optional) dz column sums -> colsum
    [xent_blocks(rows)][width] (bias-gradient partials)."""
    rows, width = dz.shape
    if loss_part is not None and loss_part.numel() < xent_blocks(rows):
        raise ValueError("loss_part needs xent_blocks(rows) entries")
    if correct is not None and (correct.dtype != torch.int32 or
                                correct.numel() < xent_blocks(rows)):
        raise ValueError("correct needs xent_blocks(rows) int32 entries")
    if colsum is not None and (colsum.dtype != torch.float32 or colsum.dim() != 2 or
                               colsum.shape[0] < xent_blocks(rows) or colsum.shape[1] < width
                               or colsum.stride(1) != 1):
        raise ValueError("colsum must be fp32 [xent_blocks(rows)][>=width]")
    if not logits.is_cuda:
        return ref.softmax_xent(logits, labels, dz, n_cls, scale, loss_part, correct,
                                XENT_ROWS_PER_BLOCK, colsum)
    _rows(logits, "logits", torch.float32)
    _rows(dz, "dz", torch.bfloat16)
    if labels.dtype != torch.int32 or labels.numel() < rows or logits.shape[0] < rows:
        raise ValueError("labels must be int32 with one entry per row")
    native().softmax_xent(_p(logits), logits.stride(0), _p(labels), _p(dz), dz.stride(0), rows,
                          n_cls, width, float(scale), _p(loss_part), _p(correct),
                          _stream(logits), _p(colsum),
                          colsum.stride(0) if colsum is not None else 0)


TAIL_MAX_CLS = 16


def tail_supported(k3: int, n3: int, n4: int, n_cls: int) -> bool:
    """Geometries the fused classifier tail (csrc/kernels/mlp_tail.hip) handles."""
    return k3 in (64, 128, 256) and n3 in (64, 128) and n4 in (64, 128) and \
        1 <= n_cls <= TAIL_MAX_CLS


def tail_blocks(rows: int) -> int:
    """Partials (workgroups) of one mlp_tail launch over ``rows`` rows."""
    if rows <= 0 or rows % 16:
        raise ValueError("mlp_tail rows must be a positive multiple of 16")
    if torch.cuda.is_available():
        return int(native().mlp_tail_blocks(rows))
    return max(1, min(NUM_CU, -(-rows // ref.TAIL_BLOCK_ROWS)))


def mlp_tail(x, w3, b3, w4, b4, labels, h3, dz4, dz3, dz2, n_cls, scale, act3="relu",
             act2="relu", loss_part=None, correct=None, cs4=None, cs3=None, cs2=None):
    """The last two layers of a narrow classifier, forward AND backward, in one launch:
    h3 = act3(x.w3^T + b3); dz4 = (softmax(h3.w4^T + b4) - onehot) * scale;
    dz3 = (dz4.w4) * act3'(h3); dz2 = (dz3.w3) * act2'(x) (GPU: dz4 columns >= 16 are not
    written -- they stay the zeros the caller allocated); bias-gradient partials
    cs4/cs3/cs2 [tail_blocks(rows)][cols] and per-block loss / correct counts.
    CPU: the unfused kernels' reference path (same contract, partials per 64-row block)."""
    rows, k3 = x.shape
    n3, n4 = w3.shape[0], w4.shape[0]
    if not tail_supported(k3, n3, n4, n_cls) or w3.shape[1] != k3 or w4.shape[1] != n3:
        raise ValueError(f"mlp_tail: unsupported geometry K3={k3} N3={n3} N4={n4} "
                         f"classes={n_cls}")
    nb = tail_blocks(rows)
    for t, name, cols in ((cs4, "cs4", n4), (cs3, "cs3", n3), (cs2, "cs2", k3)):
        if t is None or t.dtype != torch.float32 or t.dim() != 2 or t.shape[0] < nb or \
                t.shape[1] < cols or t.stride(1) != 1:
            raise ValueError(f"{name} must be fp32 [{nb}][>={cols}] row-major")
    if loss_part is None or loss_part.numel() < nb or correct is None or \
            correct.dtype != torch.int32 or correct.numel() < nb:
        raise ValueError(f"loss_part / correct (int32) need {nb} entries")
    if not x.is_cuda:
        ref.mlp_tail(x, w3, b3, w4, b4, labels, h3, dz4, dz3, dz2, n_cls, scale, _act(act3),
                     _act(act2), loss_part, correct, cs4, cs3, cs2, nb)
        return
    for t, name in ((x, "x"), (w3, "w3"), (w4, "w4"), (h3, "h3"), (dz4, "dz4"), (dz3, "dz3"),
                    (dz2, "dz2")):
        _rows(t, name, torch.bfloat16)
    if labels.dtype != torch.int32 or labels.numel() < rows:
        raise ValueError("labels must be int32 with one entry per row")
    native().mlp_tail(_p(x), x.stride(0), _p(w3), w3.stride(0), _p(b3), _p(w4), w4.stride(0),
                      _p(b4), _p(labels), _p(h3), h3.stride(0), _p(dz4), dz4.stride(0),
                      _p(dz3), dz3.stride(0), _p(dz2), dz2.stride(0), _p(loss_part),
                      _p(correct), _p(cs4), cs4.stride(0), _p(cs3), cs3.stride(0), _p(cs2),
                      cs2.stride(0), rows, k3, n3, n4, n_cls, float(scale), _act(act3),
                      _act(act2), _stream(x))


def softmax_rows(logits, out, n_cls, labels=None, pred=None, correct=None):
    rows = logits.shape[0]
    if not logits.is_cuda:
        return ref.softmax_rows(logits, out, n_cls, labels, pred, correct)
    _rows(logits, "logits", torch.float32)
    if out is not None:
        _rows(out, "out", torch.float32)
    native().softmax_rows(_p(logits), logits.stride(0), _p(out),
                          out.stride(0) if out is not None else 0, rows, n_cls, _p(labels),
                          _p(pred), _p(correct), _stream(logits))


def colsum_partial(x, part, n_part=None):
    """part[n_part][cols] = partial column sums of x (row blocks)."""
    rows, cols = x.shape
    n_part = n_part or part.shape[0]
    if not x.is_cuda:
        return ref.colsum_partial(x, part, n_part)
    _rows(x, "x", torch.bfloat16)
    if part.dtype != torch.float32 or not part.is_contiguous() or part.numel() < n_part * cols:
        raise ValueError("part must be contiguous fp32 [n_part][cols]")
    native().colsum_partial(_p(x), x.stride(0), rows, cols, n_part, _p(part), _stream(x))


def reduce_slabs(src, n_src, stride, n, out, scale=1.0, accumulate=False):
    """out[:n] (+)= scale * sum_s src_flat[s*stride : s*stride+n]."""
    if not src.is_cuda:
        return ref.reduce_slabs(src, n_src, stride, n, out, scale, accumulate)
    if src.dtype != torch.float32 or out.dtype != torch.float32:
        raise TypeError("reduce_slabs works on fp32")
    if not (src.is_contiguous() and out.is_contiguous()):
        raise ValueError("reduce_slabs needs contiguous buffers")
    if (n_src - 1) * stride + n > src.numel() or out.numel() < n:
        raise ValueError("reduce_slabs range out of bounds")
    native().reduce_slabs(_p(src), stride, n_src, n, float(scale), _p(out), int(accumulate),
                          _stream(src))


def reduce_multi(jobs, sgd=None, max_blocks: int = 0):
    """Several reduce_slabs in ONE launch. jobs: iterable of
    (src, n_src, stride, n, out, scale, accumulate) with reduce_slabs' meaning; the results are
    bitwise identical to running reduce_slabs on each job.

    ``sgd`` (GPU): dict(grad=flat fp32 gradient the outputs live in, master=, mom=None,
    shadow=None, lr=, momentum=0, weight_decay=0, lr_dev=None) -- the same launch also applies
    the SGD step to every reduced element (bitwise equal to a following sgd_update over them).
    With adam=True (and v=, betas=, eps=, decoupled=, step_dev= as for adam_update; mom = the
    first moment) it applies the Adam / AdamW step instead, bitwise equal to adam_update; the
    caller advances step_dev afterwards.

    A job may carry an 8th element ``wt`` (GPU, fused update with a shadow only): the bf16
    W^T[cols][rows] of the layer whose [rows][cols] weight gradient the job reduces; the update
    writes it too (bitwise the transpose of the refreshed shadow).

    ``max_blocks`` (GPU, > 0): cap the launch at that many workgroups (each loops over the
    blocks; same results) -- for a reduction that runs beside other kernels."""
    jobs = [tuple(j) + (None,) * (8 - len(j)) for j in jobs]
    if not jobs:
        return
    if not jobs[0][0].is_cuda:
        for (src, n_src, stride, n, out, scale, acc, _wt) in jobs:
            ref.reduce_slabs(src, n_src, stride, n, out, scale, acc)
        if sgd is not None and sgd.get("adam"):
            adam_update(sgd["master"], sgd["grad"], sgd["mom"], sgd["v"], sgd.get("shadow"),
                        lr=sgd["lr"], betas=sgd["betas"], eps=sgd["eps"],
                        weight_decay=sgd.get("weight_decay", 0.0),
                        decoupled=sgd.get("decoupled", False), step=sgd.get("step", 1),
                        lr_dev=sgd.get("lr_dev"), step_dev=sgd.get("step_dev"))
        elif sgd is not None:
            sgd_update(sgd["master"], sgd["grad"], sgd.get("mom"), sgd.get("shadow"),
                       lr=sgd["lr"], momentum=sgd.get("momentum", 0.0),
                       weight_decay=sgd.get("weight_decay", 0.0), lr_dev=sgd.get("lr_dev"))
        return
    packed = []
    for (src, n_src, stride, n, out, scale, acc, wt) in jobs:
        if src.dtype != torch.float32 or out.dtype != torch.float32:
            raise TypeError("reduce_multi works on fp32")
        if not (src.is_contiguous() and out.is_contiguous()):
            raise ValueError("reduce_multi needs contiguous buffers")
        if (n_src - 1) * stride + n > src.numel() or out.numel() < n:
            raise ValueError("reduce_multi range out of bounds")
        if wt is not None:
            if sgd is None or sgd.get("shadow") is None:
                raise ValueError("reduce_multi: W^T output needs the fused update with a shadow")
            if wt.dtype != torch.bfloat16 or wt.dim() != 2 or not wt.is_contiguous() or \
                    wt.numel() != n or wt.shape[0] % 4:
                raise ValueError("reduce_multi: W^T must be contiguous bf16 [cols][rows] of the "
                                 "job's n elements, cols a multiple of 4")
        packed.append((_p(src), int(stride), int(n_src), int(n), _p(out), float(scale),
                       int(acc), _p(wt), int(wt.shape[0]) if wt is not None else 0))
    if sgd is None:
        native().reduce_multi(packed, _stream(jobs[0][0]), max_blocks=int(max_blocks))
        return
    g, m = sgd["grad"], sgd["master"]
    adam = bool(sgd.get("adam"))
    if adam and (sgd.get("mom") is None or sgd.get("v") is None):
        raise ValueError("fused Adam needs both moment buffers")
    for t in (m, sgd.get("mom"), sgd.get("v")):
        if t is not None and (t.dtype != torch.float32 or t.numel() != g.numel()):
            raise ValueError("fused SGD buffers must match the flat gradient")
    sh = sgd.get("shadow")
    if sh is not None and (sh.dtype != torch.bfloat16 or sh.numel() != g.numel()):
        raise ValueError("fused SGD shadow must be bf16 like the flat gradient")
    native().reduce_multi(packed, _stream(jobs[0][0]), grad_base=_p(g), master=_p(m),
                          mom=_p(sgd.get("mom")), shadow=_p(sh), lr=float(sgd["lr"]),
                          mu=float(sgd.get("momentum", 0.0)),
                          wd=float(sgd.get("weight_decay", 0.0)), lr_dev=_p(sgd.get("lr_dev")),
                          max_blocks=int(max_blocks), **(_adam_args(sgd) if adam else {}))


def _adam_args(sgd: dict) -> dict:
    b1, b2 = sgd["betas"]
    step = int(sgd.get("step", 1))
    sd = sgd.get("step_dev")
    if sd is not None and sd.dtype != torch.int32:
        raise TypeError("step_dev must be int32")
    return dict(adam=1, v=_p(sgd["v"]), b1=float(b1), b2=float(b2), eps=float(sgd["eps"]),
                decoupled=int(bool(sgd.get("decoupled", False))), step_dev=_p(sd),
                db1=float(b1), db2=float(b2), bc1=float(1.0 / (1.0 - b1 ** step)),
                bc2=float(1.0 / (1.0 - b2 ** step)))


def sgd_update(p, g, mom=None, shadow=None, lr=0.01, momentum=0.0, weight_decay=0.0,
               lr_dev=None):
    """Fused SGD over flat buffers. ``lr_dev`` (fp32 [1] device tensor): read the learning
    rate from device memory instead (replayable under an LR schedule)."""
    if not p.is_cuda:
        if lr_dev is not None:
            lr = float(lr_dev[0])
        return ref.sgd_update(p, g, mom, shadow, lr, momentum, weight_decay)
    n = p.numel()
    if g.numel() != n or (mom is not None and mom.numel() != n) or (
            shadow is not None and shadow.numel() != n):
        raise ValueError("sgd buffers must have equal sizes")
    native().sgd_update(_p(p), _p(g), _p(mom if momentum else None), _p(shadow), n, float(lr),
                        float(momentum), float(weight_decay), _stream(p), lr_dev=_p(lr_dev))


def adam_update(p, g, m, v, shadow=None, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                weight_decay=0.0, decoupled=False, step=1, lr_dev=None, step_dev=None):
    """Fused Adam/AdamW. ``step`` is the 1-based step of this update; with ``step_dev`` (int32
    [1] device tensor holding the number of PREVIOUS updates) and ``lr_dev`` the bias
    corrections and learning rate are taken from device memory (replayable); advance the
    counter with :func:`step_advance` after the update."""
    b1, b2 = betas
    if not p.is_cuda:
        if lr_dev is not None:
            lr = float(lr_dev[0])
        if step_dev is not None:
            step = int(step_dev[0]) + 1
        return ref.adam_update(p, g, m, v, shadow, lr, b1, b2, eps, weight_decay, decoupled,
                               1.0 / (1.0 - b1 ** step), 1.0 / (1.0 - b2 ** step))
    bc1 = 1.0 / (1.0 - b1 ** step)
    bc2 = 1.0 / (1.0 - b2 ** step)
    n = p.numel()
    if any(t.numel() != n for t in (g, m, v)):
        raise ValueError("adam buffers must have equal sizes")
    if step_dev is not None and step_dev.dtype != torch.int32:
        raise TypeError("step_dev must be int32")
    native().adam_update(_p(p), _p(g), _p(m), _p(v), _p(shadow), n, float(lr), float(b1),
                         float(b2), float(eps), float(weight_decay), int(decoupled), float(bc1),
                         float(bc2), _stream(p), lr_dev=_p(lr_dev), step_dev=_p(step_dev),
                         db1=float(b1), db2=float(b2))


def step_advance(step_dev):
    """step_dev += 1 on the device (after a device-step optimizer update)."""
    if not step_dev.is_cuda:
        step_dev += 1
        return
    native().step_advance(_p(step_dev), _stream(step_dev))


def pack_bf16(src, out):
    """fp32 [rows][cols] -> padded bf16 out [rows_p][cols_p] (zero padding)."""
    rows, cols = src.shape
    rows_p, cols_p = out.shape
    if not out.is_cuda:
        return ref.pack_bf16(src, out)
    if src.dtype != torch.float32 or out.dtype != torch.bfloat16:
        raise TypeError("pack_bf16: fp32 -> bf16")
    if src.stride(1) != 1 or out.stride(1) != 1:
        raise ValueError("pack_bf16 needs row-major tensors")
    native().pack_bf16(_p(src), src.stride(0), rows, cols, _p(out), out.stride(0), rows_p, cols_p,
                       _stream(out))


def bias_act_cast(x, bias, y, act="relu"):
    """y (bf16) = act(x (fp32) + bias): a row-parallel layer's epilogue after its all-reduce."""
    rows, cols = y.shape
    if not x.is_cuda:
        v = x[:rows, :cols] + (bias[:cols] if bias is not None else 0.0)
        y.copy_(ref.act_fwd(v, _act(act)).to(torch.bfloat16))
        return y
    _rows(x, "x", torch.float32)
    _rows(y, "y", torch.bfloat16)
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() < cols):
        raise ValueError("bias must be fp32 with >= cols entries")
    native().bias_act_cast(_p(x), x.stride(0), _p(bias), _act(act), _p(y), y.stride(0), rows,
                           cols, _stream(x))
    return y


def unpack_bf16(src, out):
    rows, cols = out.shape
    if not src.is_cuda:
        out.copy_(src[:rows, :cols].float())
        return
    native().unpack_bf16(_p(src), src.stride(0), rows, cols, _p(out), out.stride(0),
                         _stream(src))
