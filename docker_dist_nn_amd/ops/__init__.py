from .kernels import (STREAMK_WG, linear_fwd_xent, xent_tiles, linear_wgrad_streamk, streamk_partial_elems, streamk_tiles,
                      KMAJ, MNMAJ, adam_update, colsum_partial, dgrad_tiles, gemm, linear_dgrad, linear_fwd,
                      linear_wgrad, pack_bf16, pick_splits, pick_tiles, reduce_slabs, sgd_update,
                      softmax_rows, softmax_xent, unpack_bf16, xent_blocks)

__all__ = ["STREAMK_WG", "linear_fwd_xent", "xent_tiles", "linear_wgrad_streamk", "streamk_partial_elems", "streamk_tiles", "KMAJ", "MNMAJ", "adam_update", "colsum_partial", "dgrad_tiles", "gemm", "linear_dgrad",
           "linear_fwd", "linear_wgrad", "pack_bf16", "pick_splits", "pick_tiles",
           "reduce_slabs", "sgd_update", "softmax_rows", "softmax_xent", "unpack_bf16",
           "xent_blocks"]
