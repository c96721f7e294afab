"""ctypes binding of libensvs.so (the gfx950 C ABI declared in include/ensvs.h).

The product path has no fallback: if the shared library is missing or cannot
be loaded, importing anything that launches a kernel raises immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The training step runs its branches on concurrent HIP streams (engine.Branches), one
# hardware queue each under HIP's default GPU_MAX_HW_QUEUES=4 (what the GPU boxes export).
# No queue count is forced: 8 queues measured 15.9 vs 14.6 ms per 30 x 1024 step in round 4
# (profiles/r4_defer_params_ab.txt; round 2's schedule had measured the opposite, 20.6 vs
# 21.0-21.4 ms, before the branch start order and the recurrence LDS reservation).
# ENSVS_LIB: another in-tree build of the same ABI, for A/B timing of a kernel change
# (tools/ab_lib.sh); the default is the package's own libensvs.so
LIB_PATH = os.environ.get("ENSVS_LIB") or os.path.join(_HERE, "libensvs.so")

c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_float = ctypes.c_float
c_double = ctypes.c_double
c_vp = ctypes.c_void_p

STATUS = {0: "OK", 1: "E_SHAPE", 2: "E_DTYPE", 3: "E_HIP", 4: "E_ARG"}

PAD_ZERO, PAD_REFLECT, PAD_REPLICATE = 0, 1, 2
DT_F32, DT_BF16 = 0, 1
EPI_PLAIN, EPI_GATE, EPI_RESSKIP, EPI_GATE_BWD, EPI_ADDSCALE, EPI_RELU_MASK = 0, 1, 2, 3, 4, 5
EPI_GATE_TS = 6
EPI_NONE = 7  # measurement only: the GEMM main loop without any output
EPI_AUX0_BF16, EPI_AUX1_BF16 = 256, 512  # flags or-ed into epi (include/ensvs.h)
ACT_RELU, ACT_SIGMOID = 1, 2


class ConvSeg(ctypes.Structure):
    _fields_ = [
        ("x", c_vp), ("radd", c_vp), ("pd", c_vp), ("wofs", c_ll),
        ("ld", c_int), ("K", c_int), ("taps", c_int), ("dil", c_int), ("shift0", c_int),
        ("pad", c_int), ("radd_ld", c_int), ("Tin", c_int), ("Kp", c_int), ("pd_dil", c_int),
    ]


class PackDesc(ctypes.Structure):
    _fields_ = [
        ("src", c_vp), ("src2", c_vp), ("dst", c_vp),
        ("sn", c_ll), ("sk", c_ll), ("sj", c_ll),
        ("N", c_int), ("K", c_int), ("taps", c_int), ("Npad", c_int), ("Kp", c_int),
        ("perm_c", c_int), ("flip", c_int), ("transpose", c_int), ("dtype", c_int),
        ("scale", c_float), ("ldk", c_int), ("tile0", c_int),
    ]


# name -> argtypes (every entry point returns int status)
SIGNATURES = {
    "ensvs_conv_gemm": [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int,
                        c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_float, c_int, c_vp],
    "ensvs_conv_gemm_bf16a": [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int,
                              c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_float, c_int,
                              c_int, c_vp, c_ll, c_vp],
    "ensvs_conv_wgrad_bf16": [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_int, c_int, c_vp, c_vp, c_ll, c_ll, c_ll, c_int,
                              c_float, c_vp],
    "ensvs_conv_gemm_bf16a_out": [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                  c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_float,
                                  c_int, c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int, c_vp,
                                  c_ll, c_vp],
    "ensvs_set_big_tile": [c_int, c_int],
    "ensvs_set_p8": [c_int], "ensvs_set_p8_min_tiles": [c_int], "ensvs_set_p8h": [c_int],
    "ensvs_set_dual_small": [c_int],
    "ensvs_set_gbw_dma": [c_int],
    "ensvs_set_wgrad_big": [c_int],
    "ensvs_set_small": [c_int],
    "ensvs_set_recurrence_exclusive": [c_int],
    "ensvs_note_mask": [c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_filtfilt_multi": [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_vp],
    "ensvs_f0_from_lf0": [c_vp, c_int, c_vp, c_int, c_int, c_float, c_int, c_vp, c_vp],
    "ensvs_usf_block": [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_ll, c_int, c_vp, c_vp,
                        c_int, c_float, c_int, c_vp, c_int, c_vp],
    "ensvs_tile_colsum": [c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp],
    "ensvs_cast_bf16": [c_vp, c_int, c_vp, c_int, c_int, c_ll, c_int, c_vp, c_int, c_vp],
    "ensvs_conv_wgrad": [c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_ll, c_ll, c_ll, c_int,
                         c_float, c_int, c_vp],
    "ensvs_pack_weights": [c_vp, c_int, c_int, c_vp],
    "ensvs_pack_weights_tiled": [c_vp, c_int, c_int, c_vp],
    "ensvs_colsum_batch": [c_vp, c_int, c_vp, c_ll, c_vp],
    "ensvs_colsum_batch_part_floats": [c_vp, c_int],
    "ensvs_colsum_once": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_float, c_vp, c_int, c_vp,
                          c_vp, c_int, c_int, c_vp],
    "ensvs_colsum": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_float, c_vp, c_int, c_vp, c_int,
                     c_int, c_vp],
    "ensvs_lstm_fwd": [c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp,
                       c_vp],
    "ensvs_lstm_bwd_work_floats": [c_int, c_int],
    "ensvs_lstm_set_step": [c_int],
    "ensvs_lstm_bwd": [c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int,
                       c_vp, c_ll, c_vp],
    "ensvs_lstm_mfma_supported": [c_int],
    "ensvs_lstm_mfma_pack": [c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_lstm_mfma_fwd": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp,
                            c_int, c_vp],
    "ensvs_lstm_mfma_bwd": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp,
                            c_int, c_vp, c_vp],
    "ensvs_lstm_coop_supported": [c_int, c_int],
    "ensvs_lstm_coop_work_bytes": [c_int, c_int],
    "ensvs_lstm_coop_tile_seqs": [c_int, c_int],
    "ensvs_lstm_coop_set_tile_seqs": [c_int],
    "ensvs_ardec_coop_tile_seqs": [c_int, c_int],
    "ensvs_ardec_coop_set_tile_seqs": [c_int],
    "ensvs_lstm_coop_pack": [c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_lstm_coop_fwd": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp,
                            c_ll, c_vp],
    "ensvs_lstm_coop_bwd": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp,
                            c_ll, c_vp],
    "ensvs_lstm_coop_fwd_ex": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp,
                               c_vp, c_int, c_vp, c_ll, c_vp],
    "ensvs_lstm_coop_bwd_ex": [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int,
                               c_vp, c_int, c_vp, c_vp, c_ll, c_vp],
    "ensvs_ardec_pack": [c_vp, c_int, c_vp, c_vp, c_vp],
    "ensvs_ardec_fwd": [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                        c_vp, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp,
                        c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ensvs_ardec_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int,
                        c_float, c_float, c_float, c_float, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ensvs_ardec_coop_supported": [c_int, c_int],
    "ensvs_ardec_coop_work_bytes": [c_int, c_int],
    "ensvs_wgrad_reduce_batch": [c_vp, c_int, c_vp],
    "ensvs_coop_set_error_word": [c_vp],
    "ensvs_coop_set_error_word_dev": [c_int, c_vp],
    "ensvs_coop_error_word": [c_int],
    "ensvs_coop_set_timeout_us": [c_ll],
    "ensvs_coop_inject_fault": [c_int],
    "ensvs_ardec_coop_pack": [c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_ardec_coop_fwd": [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                             c_vp, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_float,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp],
    "ensvs_ardec_coop_bwd": [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int,
                             c_float, c_float, c_float, c_float, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_ll, c_vp],
    "ensvs_downsample_fwd": [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp,
                             c_vp, c_int, c_int, c_vp, c_int, c_vp],
    "ensvs_downsample_bwd": [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_int,
                             c_int, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp],
    "ensvs_phoneme_ids": [c_vp, c_int, c_ll, c_int, c_int, c_vp, c_vp],
    "ensvs_embed_add": [c_vp, c_int, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
    "ensvs_embed_bwd": [c_vp, c_int, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_vp],
    "ensvs_embed_bwd_workspace": [c_ll, c_int, c_int],
    "ensvs_spk_scatter": [c_vp, c_int, c_int, c_vp, c_vp, c_vp],
    "ensvs_gather_rows": [c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_bn_finalize": [c_vp, c_vp, c_int, c_int, c_ll, c_float, c_vp, c_vp, c_vp, c_float, c_int,
                          c_vp],
    "ensvs_bn_stats_part_floats": [c_ll, c_int, c_ll],
    "ensvs_bn_stats": [c_vp, c_int, c_ll, c_int, c_ll, c_vp, c_ll, c_float, c_vp, c_vp, c_vp, c_vp,
                       c_vp, c_float, c_int, c_vp, c_vp],
    "ensvs_bn_apply_relu": [c_vp, c_int, c_ll, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                            c_vp, c_int, c_vp],
    "ensvs_bn_bwd": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp,
                     c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp],
    "ensvs_bn_bwd_frozen": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
    "ensvs_sinusoidal": [c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_mish_fwd": [c_vp, c_vp, c_ll, c_vp],
    "ensvs_mish_bwd": [c_vp, c_vp, c_vp, c_ll, c_vp],
    "ensvs_q_sample": [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_float,
                       c_vp, c_int, c_vp],
    "ensvs_p_sample": [c_vp, c_vp, c_vp, c_ll, c_float, c_float, c_float, c_float, c_float, c_vp],
    "ensvs_p_sample_bf16": [c_vp, c_vp, c_vp, c_ll, c_int, c_float, c_float, c_float, c_float,
                            c_float, c_vp, c_int, c_vp],
    "ensvs_masked_l1": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int,
                        c_float, c_float, c_vp, c_vp, c_vp],
    "ensvs_lf0_interaction": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_int, c_int,
                              c_float, c_float, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ensvs_l2norm": [c_vp, c_ll, c_vp, c_vp, c_vp],
    "ensvs_l2norm_chk": [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp],
    "ensvs_poison_on_error": [c_vp, c_vp, c_vp],
    "ensvs_adam": [c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_float, c_float, c_float, c_float, c_float,
                   c_float, c_float, c_vp],
    "ensvs_adam_step": [c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_float, c_double, c_double, c_float,
                        c_vp, c_vp],
    "ensvs_rng_advance": [c_vp],
    "ensvs_copy_cols": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_vp],
    "ensvs_regroup_cols": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_int, c_int, c_vp],
    "ensvs_axpy": [c_vp, c_vp, c_float, c_ll, c_vp],
    "ensvs_axpy_strided": [c_vp, c_ll, c_vp, c_ll, c_float, c_int, c_int, c_vp],
    "ensvs_axpy_blocks2d": [c_vp, c_ll, c_ll, c_vp, c_ll, c_ll, c_float, c_int, c_int, c_int,
                            c_vp],
    "ensvs_res_bias_grad": [c_vp, c_int, c_int, c_vp, c_ll, c_float, c_vp],
    "ensvs_axpby": [c_vp, c_float, c_vp, c_float, c_ll, c_vp],
    "ensvs_axpby_to": [c_vp, c_vp, c_float, c_vp, c_float, c_ll, c_vp],
    "ensvs_axpby_to_bf16": [c_vp, c_vp, c_vp, c_float, c_vp, c_float, c_ll, c_vp],
    "ensvs_mul": [c_vp, c_vp, c_ll, c_vp],
    "ensvs_mul_out": [c_vp, c_vp, c_vp, c_ll, c_vp],
    "ensvs_relu_mask": [c_vp, c_vp, c_vp, c_vp, c_ll, c_vp],
    "ensvs_reflect_fold": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "ensvs_randn": [c_vp, c_ll, ctypes.c_ulonglong, c_vp],
    "ensvs_dropout_mask": [c_vp, c_ll, c_float, ctypes.c_ulonglong, c_vp],
    "ensvs_randint": [c_vp, c_ll, c_ll, ctypes.c_ulonglong, c_vp],
    "ensvs_weight_norm": [c_vp, c_vp, c_int, c_int, c_vp, c_ll, c_ll, c_vp],
    "ensvs_usf_upsample": [c_vp, c_int, c_int, c_int, c_int, c_int, c_float, c_vp, c_vp, c_vp],
    "ensvs_usf_dfactor": [c_vp, c_int, c_int, c_int, c_double, c_double, c_vp, c_vp],
    "ensvs_usf_source_workspace": [c_int, c_int, c_int],
    "ensvs_usf_source": [c_vp, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_vp,
                         c_vp, c_vp, c_vp, c_int, c_vp],
    "ensvs_usf_mix": [c_vp, c_vp, c_vp, c_vp, c_ll, c_int, c_vp],
    "ensvs_mdn_log_softmax": [c_vp, c_ll, c_int, c_int, c_int, c_vp],
    "ensvs_mdn_log_softmax_bwd": [c_vp, c_vp, c_ll, c_int, c_int, c_int, c_vp],
    "ensvs_mdn_loss": [c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_int, c_int, c_int, c_float,
                       c_float, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "ensvs_mdn_most_probable": [c_vp, c_vp, c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp],
    "ensvs_layer_norm_fwd": [c_vp, c_int, c_ll, c_int, c_vp, c_vp, c_float, c_vp, c_int, c_vp,
                             c_vp, c_vp],
    "ensvs_layer_norm_bwd": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp,
                             c_int, c_vp, c_vp],
    "ensvs_masked_mean": [c_vp, c_vp, c_ll, c_vp, c_vp, c_vp],
    "ensvs_masked_mean_bwd": [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp],
    "ensvs_bgemm": [c_vp, c_ll, c_ll, c_ll, c_ll, c_vp, c_ll, c_ll, c_ll, c_ll, c_vp, c_ll, c_ll,
                    c_ll, c_ll, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_vp],
    "ensvs_bgemm_bf16": [c_vp, c_ll, c_ll, c_ll, c_ll, c_vp, c_ll, c_ll, c_ll, c_ll, c_vp, c_ll,
                         c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                         c_vp],
    "ensvs_div": [c_vp, c_int, c_vp, c_int, c_ll, c_int, c_float, c_vp],
    "ensvs_attn_softmax": [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int,
                           c_vp, c_vp, c_vp],
    "ensvs_attn_relv": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "ensvs_attn_band_dot": [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "ensvs_attn_table_grad_workspace": [c_int, c_int],
    "ensvs_attn_table_grad": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp,
                              c_int, c_vp],
    "ensvs_attn_softmax_bwd": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp],
    "ensvs_attn_band_rows": [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "ensvs_mask_rows": [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "ensvs_stride_rows": [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_vp],
    "ensvs_dwdown_fwd": [c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "ensvs_dwdown_bwd": [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int,
                         c_int, c_vp],
    "ensvs_gv_scale": [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp],
    "ensvs_world_lf0": [c_vp, c_int, c_vp, c_int, c_int, c_float, c_float, c_vp, c_vp],
    "ensvs_filtfilt": [c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp],
    "ensvs_bap_post": [c_vp, c_int, c_int, c_int, c_int, c_int, c_vp],
    "ensvs_scale_cols": [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp],
}

# entry points returning a value instead of a status code
RESTYPES = {"ensvs_embed_bwd_workspace": c_ll, "ensvs_usf_source_workspace": c_ll,
            "ensvs_attn_table_grad_workspace": c_ll, "ensvs_lstm_bwd_work_floats": c_ll,
            "ensvs_lstm_coop_work_bytes": c_ll, "ensvs_lstm_coop_supported": ctypes.c_int,
            "ensvs_lstm_mfma_supported": ctypes.c_int,
            "ensvs_ardec_coop_work_bytes": c_ll, "ensvs_ardec_coop_supported": ctypes.c_int,
            "ensvs_coop_error_word": c_vp, "ensvs_colsum_batch_part_floats": c_ll,
            "ensvs_bn_stats_part_floats": c_ll}

_lib = None


def load():
    """Load libensvs.so once; raise (never fall back) when it is unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"ensvs: {LIB_PATH} not found — build it with `make` (or __graft_entry__.build()); "
                "there is no CPU fallback on the product path")
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, c_int)
        _lib = lib
    return _lib


def call(name, *args):
    status = getattr(load(), name)(*args)
    if status != 0:
        raise RuntimeError(f"{name} failed with {STATUS.get(status, status)}")


def query(name, *args):
    """Call a size-query entry point (RESTYPES) and return its value."""
    return getattr(load(), name)(*args)


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()
