from .kernels import (GEMV_MAX_ROWS, KMAJ, MNMAJ, STREAMK_WG, adam_update, blas_gemm,
                      relu_mask_bits, FragMask, frag_mask_tiles,
                      colsum_partial, dact_colsum, dequant_rows_fp8, quant_rows_fp8,
                      dgrad_tiles, gemm, gemv, linear_dgrad, linear_fwd, linear_fwd_xent,
                      linear_wgrad, linear_wgrad_group, linear_wgrad_streamk, mlp_tail, pack_bf16, pick_splits, pick_tiles,
                      reduce_multi, reduce_slabs, sgd_update, softmax_rows, softmax_xent,
                      step_advance, streamk_partial_elems, streamk_tiles, tail_blocks,
                      tail_supported, transpose_bf16, transpose_multi, unpack_bf16, bias_act_cast, wgrad_config, xent_blocks,
                      xent_tiles)

__all__ = ["GEMV_MAX_ROWS", "KMAJ", "MNMAJ", "STREAMK_WG", "adam_update", "blas_gemm",
           "relu_mask_bits", "FragMask", "frag_mask_tiles",
           "colsum_partial", "dact_colsum", "dequant_rows_fp8", "quant_rows_fp8",
           "dgrad_tiles", "gemm", "gemv", "linear_dgrad", "linear_fwd", "linear_fwd_xent",
           "linear_wgrad", "linear_wgrad_group", "linear_wgrad_streamk", "mlp_tail", "pack_bf16", "pick_splits", "pick_tiles",
           "reduce_multi", "reduce_slabs", "sgd_update", "softmax_rows", "softmax_xent",
           "step_advance", "streamk_partial_elems", "streamk_tiles", "tail_blocks", "tail_supported",
           "transpose_bf16", "transpose_multi", "unpack_bf16", "bias_act_cast", "wgrad_config", "xent_blocks", "xent_tiles"]
