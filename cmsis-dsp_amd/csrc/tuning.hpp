// Build-time tuning knobs of the kernels, in one place (VERDICT r3 Weak #10).  Every default is
// the measured best (DESIGN.md §4 gives the sweeps); a non-default value is an A/B experiment:
// `make DEFS="-DMI355X_X=..."` or tools/build_variant.sh, and arm_mi355x_version() lists it, so a
// bench line always names the kernels it timed.
#pragma once


// ---- cfft_f32.hip
#ifndef MI355X_N1024_WAVES
#define MI355X_N1024_WAVES 1
#endif
#ifndef MI355X_N1024_TWLDS  // 1: stage twiddles from a workgroup LDS copy at each use, 0: in registers
#define MI355X_N1024_TWLDS 0
#endif
#ifndef MI355X_N1024_T
#define MI355X_N1024_T 4
#endif
#ifndef MI355X_N1024_WPB
#define MI355X_N1024_WPB 8
#endif
#ifndef MI355X_N1024_LAT      // drop-in batch-1 N = 1024: the 2-wave latency-shaped kernel
#define MI355X_N1024_LAT 1
#endif
#ifndef MI355X_N1024_SPLIT
#define MI355X_N1024_SPLIT 1
#endif
#ifndef MI355X_NT
#define MI355X_NT 1
#endif
#ifndef MI355X_N4096_WAVES
#define MI355X_N4096_WAVES 1
#endif
#ifndef MI355X_N4096_T
#define MI355X_N4096_T 8
#endif
#ifndef MI355X_F32_N4096
#define MI355X_F32_N4096 1
#endif
#ifndef MI355X_N512_T
#define MI355X_N512_T 2
#endif
#ifndef MI355X_N512_WPB
#define MI355X_N512_WPB 8
#endif
#ifndef MI355X_F32_N512
#define MI355X_F32_N512 1
#endif
#ifndef MI355X_N2048_T
#define MI355X_N2048_T 2
#endif
#ifndef MI355X_N2048_WPB
#define MI355X_N2048_WPB 4
#endif
#ifndef MI355X_F32_N2048
#define MI355X_F32_N2048 1
#endif

// ---- cfft_fixed.hip
#ifndef MI355X_FX_Q31_SLOTS
#define MI355X_FX_Q31_SLOTS 6912
#endif
#ifndef MI355X_FX_WAVES
#define MI355X_FX_WAVES 1     // minimum waves per SIMD the register allocation must allow
#endif
#ifndef MI355X_FX_TW3_LDS
#define MI355X_FX_TW3_LDS 0
#endif
#ifndef MI355X_FX_TW4_LDS
#define MI355X_FX_TW4_LDS 0
#endif
#ifndef MI355X_FX_PF
#define MI355X_FX_PF 1
#endif
#ifndef MI355X_FX_Q15_PFD
#define MI355X_FX_Q15_PFD 2
#endif
#ifndef MI355X_FXQ15_SLOTS
#define MI355X_FXQ15_SLOTS 4351   // LDS words of the q15 kernel (more: fewer workgroups per CU)
#endif
#ifndef MI355X_FXQ15_TW34_LDS
#define MI355X_FXQ15_TW34_LDS 0
#endif
#ifndef MI355X_FXQ15_WAVES
#define MI355X_FXQ15_WAVES 1
#endif

// ---- cfft_fixed_r16.hip
#ifndef MI355X_FXR_T
#define MI355X_FXR_T 8
#endif

// ---- fir.hip
#ifndef MI355X_FIR_SCHED_BARRIER
#define MI355X_FIR_SCHED_BARRIER 1
#endif
#ifndef MI355X_FIR_IPW
#define MI355X_FIR_IPW 16
#endif
#ifndef MI355X_FIR_F32_WAVES
#define MI355X_FIR_F32_WAVES(R) ((R) == 16 ? 5 : 8)   // minimum waves per SIMD the allocation must allow
#endif
#ifndef MI355X_FIR_F32_FMA_WAVES
#define MI355X_FIR_F32_FMA_WAVES 4                   // FMA: + 8 coefficient and 4 tap-staging VGPRs
#endif
#ifndef MI355X_FIR_Q7_MFMA      // arm_fir_q7 (numTaps <= 157, >= 256 items) on the i8 MFMA (fir_mfma.hip)
#define MI355X_FIR_Q7_MFMA 1
#endif
#ifndef MI355X_FIR_Q31_MFMA     // arm_fir_q31 (numTaps <= 161, >= 256 items) on the i8 MFMA (fir_mfma.hip)
#define MI355X_FIR_Q31_MFMA 1
#endif
#ifndef MI355X_FIR_FAST_Q15_MFMA   // arm_fir_fast_q15 on the same kernel (modular epilogue)
#define MI355X_FIR_FAST_Q15_MFMA 1
#endif
#ifndef MI355X_FIR_Q15_MFMA     // arm_fir_q15 (even numTaps <= 160, >= 256 items) on the i8 MFMA (fir_mfma.hip)
#define MI355X_FIR_Q15_MFMA 1
#endif
#ifndef MI355X_FIR_Q15_WAVES
#define MI355X_FIR_Q15_WAVES 1   // minimum waves per SIMD the register allocation must allow
#endif

// ---- fir_lattice.hip
#ifndef MI355X_LAT_IPW
#define MI355X_LAT_IPW 1   // 2 / 4 measured slower (f32 211 / 220 vs 221 Gsamples/s, q31 138 / 147 vs 172)
#endif

// ---- mat_mult_fixed.hip
#ifndef MI355X_I8_SCHED
#define MI355X_I8_SCHED 10
#endif
#ifndef MI355X_I8_SCHED_V3  // the same hint in the tr_b8 kernel (q31)
#define MI355X_I8_SCHED_V3 6
#endif
#ifndef MI355X_I8_STAMPS    // diagnostic: per-workgroup phase timestamps (mat_mult_fixed.hip)
#define MI355X_I8_STAMPS 0
#endif
#ifndef MI355X_I8_B8        // q15: B staged by 8-row x column-pair threads (ds_write_b64)
#define MI355X_I8_B8 1
#endif
#ifndef MI355X_I8_SPLIT     // v2: a K step's second MFMA k-step issued under the next step's fragment reads
#define MI355X_I8_SPLIT 1
#endif
#ifndef MI355X_I8_V3
#define MI355X_I8_V3 2
#endif

// ---- mfcc_f32.hip
#ifndef MI355X_MFCC_UNROLL
#define MI355X_MFCC_UNROLL 8        // Mel / DCT dot products: loads issued 8 taps ahead
#endif

// ---- rfft_f32.hip
#ifndef MI355X_RF1024_T
#define MI355X_RF1024_T 1
#endif
#ifndef MI355X_RF1024_STRIDE // 1: a wave's transforms are W apart (W = waves in the grid), 0: consecutive
#define MI355X_RF1024_STRIDE 0
#endif
#ifndef MI355X_RF1024_TWLDS  // 1: twiddles from a workgroup LDS copy at each use, 0: held in registers
#define MI355X_RF1024_TWLDS 1
#endif
#ifndef MI355X_RF1024_WPE    // >0: amdgpu_waves_per_eu floor (register budget) of the rfft1024 kernel
#define MI355X_RF1024_WPE 0
#endif
#ifndef MI355X_RF1024_TS     // transforms per wave when p is scratch (ARM_MI355X_RFFT_P_SCRATCH)
#define MI355X_RF1024_TS 2
#endif
#ifndef MI355X_RF1024_WPB
#define MI355X_RF1024_WPB 4
#endif
#ifndef MI355X_RF1024
#define MI355X_RF1024 1
#endif

// ---- cfft_fixed_core.hpp
#ifndef MI355X_FX_Q15_PACKED
#define MI355X_FX_Q15_PACKED 1
#endif
#ifndef MI355X_FX_NT
#define MI355X_FX_NT 2
#endif
#ifndef MI355X_FX_T
#define MI355X_FX_T 8
#endif
#ifndef MI355X_FXQ15_T
#define MI355X_FXQ15_T 8
#endif

// ---- mfcc_fixed_post.hpp: magnitude steps (64 bins each) unrolled per wave
#ifndef MI355X_MQ_BIN_U
#define MI355X_MQ_BIN_U 2
#endif

// ---- cfft_fixed_r16.hip: minimum workgroups per CU of the one-launch MFCC kernel (caps its VGPRs)
#ifndef MI355X_MQF_WG
#define MI355X_MQF_WG 1
#endif
#ifndef MI355X_MQF_STAGE   // stage the Mel / DCT tables in LDS when they fit 32 KiB
#define MI355X_MQF_STAGE 1
#endif

// ---- api.cpp
#ifndef MI355X_RFFT_Q31_FUSED   // forward arm_rfft_q31 N = 8192: split fused into the inner CFFT's last pass
#define MI355X_RFFT_Q31_FUSED 1
#endif
#ifndef MI355X_RFFT_FX_R16_FUSED   // forward arm_rfft_q31 / _q15 N = 512 .. 4096: split fused into the radix-16 CFFT
#define MI355X_RFFT_FX_R16_FUSED 1
#endif
#ifndef MI355X_RFFT_FX_R16_INV_FUSED   // inverse arm_rfft_q31 / _q15 N = 512 .. 4096: merge fused into the radix-16 CFFT
#define MI355X_RFFT_FX_R16_INV_FUSED 1
#endif
#ifndef MI355X_RFFT_Q31_INV_FUSED   // inverse arm_rfft_q31 N = 8192: merge fused into the CFFT-4096 (one workgroup per CU)
#define MI355X_RFFT_Q31_INV_FUSED 1
#endif
#ifndef MI355X_RFFT_Q15_INV_FUSED   // inverse arm_rfft_q15 N = 8192: merge fused into the packed CFFT-4096
#define MI355X_RFFT_Q15_INV_FUSED 1
#endif
#ifndef MI355X_RFFT_MERGE_WAVES   // fused radix-16 inverse: minimum waves per SIMD its registers must allow
#define MI355X_RFFT_MERGE_WAVES 2
#endif
#ifndef MI355X_RFFT_MERGE_XCH   // fused radix-16 inverse, N <= 1024: X[N - e] by lane exchange instead of loads
#define MI355X_RFFT_MERGE_XCH 1
#endif
#ifndef MI355X_RFFT_MERGE_LDSX   // fused radix-16 inverse, N = 2048: X[N - e] through LDS instead of loads
#define MI355X_RFFT_MERGE_LDSX 1
#endif
#ifndef MI355X_RFFT_MERGE_BLK   // fused inverse: merged elements per pinned block
#define MI355X_RFFT_MERGE_BLK 4
#endif
#ifndef MI355X_RFFT_SPLIT_UNROLL   // fused radix-16 split: bin pairs per unrolled step
#define MI355X_RFFT_SPLIT_UNROLL 2
#endif
#ifndef MI355X_RFFT_Q15_FUSED   // ... and arm_rfft_q15
#define MI355X_RFFT_Q15_FUSED 1
#endif
#ifndef MI355X_MFCC_FX_MODE
#define MI355X_MFCC_FX_MODE 1
#endif
