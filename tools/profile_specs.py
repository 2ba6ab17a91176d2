#!/usr/bin/env python3
"""Bench command of every profiled workload (tools/profile_round.sh) and the kernel whose
launches it measures (tools/profile_collect.py).  The timed launches are the dispatches of
that kernel with the LARGEST grid: bench.py also launches it on small parity batches.
Usage: profile_specs.py <name>  -> prints the bench.py arguments."""
import sys

# name: (bench.py arguments, kernel-name substring of the dominant kernel, source unit(s) of the
# kernel(s) for the valu_issue weighting ("a|b" aligned with "a|b" kernel substrings; "" = none))
SPECS = {
    "cfft_f32_1024": ("--workload cfft_f32_1024 --no-config3 --steps 10 --warmup 3", "n1024", ""),
    "cfft_q31_4096_strong1M": ("--workload cfft_q31_4096 --scaling strong --global-batch 1048576 --steps 6 --warmup 2",
                               "fx4096", "cfft_fixed"),
    "cfft_q15_4096_strong1M": ("--workload cfft_q15_4096 --scaling strong --global-batch 1048576 --steps 6 --warmup 2",
                               "q15_4096_pk", "cfft_fixed"),
    "cfft_f32_512": ("--fftlen 512 --no-config3 --steps 10 --warmup 3", "n512", ""),
    "cfft_f32_2048": ("--fftlen 2048 --no-config3 --steps 10 --warmup 3", "n2048", ""),
    "cfft_f32_4096": ("--fftlen 4096 --no-config3 --steps 10 --warmup 3", "n4096", ""),
    "rfft_f32": ("--workload rfft_f32 --steps 10 --warmup 3", "rfft1024_fwd", ""),
    "rfft_f32_pscratch": ("--workload rfft_f32_pscratch --steps 10 --warmup 3", "rfft1024_fwd", ""),
    "rfft_q31": ("--workload rfft_q31 --steps 10 --warmup 3", "fx4096", ""),
    "rfft_q15": ("--workload rfft_q15 --steps 10 --warmup 3", "q15_4096_pk", ""),
    # fftLenReal 1024: the split fused into the radix-16 CFFT-512 (round 5)
    "rfft_q31_1024": ("--workload rfft_q31 --fftlen 1024 --steps 10 --warmup 3", "cfft_fx_r16_kernel", ""),
    "rfft_q15_1024": ("--workload rfft_q15 --fftlen 1024 --steps 10 --warmup 3", "cfft_fx_r16_kernel", ""),
    "fir_f32": ("--workload fir_f32 --steps 10 --warmup 3", "fir_f32_kernel", ""),
    "fir_f32_fma": ("--workload fir_f32_fma --steps 10 --warmup 3", "fir_f32_kernel", ""),
    "fir_q15": ("--workload fir_q15 --steps 10 --warmup 3", "fir_q15_mfma", "fir_mfma"),
    "fir_q31": ("--workload fir_q31 --steps 10 --warmup 3", "fir_q31_mfma", "fir_mfma"),
    "fir_fast_q15": ("--workload fir_fast_q15 --steps 10 --warmup 3", "fir_q15_mfma", "fir_mfma"),
    "fir_fast_q31": ("--workload fir_fast_q31 --steps 10 --warmup 3", "fir_q31_kernel", "fir"),
    "conv_f32": ("--workload conv_f32 --steps 10 --warmup 3", "fir_f32_kernel", ""),
    "mfcc_f32": ("--workload mfcc_f32 --steps 10 --warmup 3", "mfcc_fused", ""),
    # two launches per step: the MFCC front end fused into the radix-16 CFFT, then post (summed)
    "mfcc_q31": ("--workload mfcc_q31 --steps 10 --warmup 3", "mfcc_q31_post|cfft_fx_r16_kernel", "mfcc_fixed|cfft_fixed_r16"),
    "mfcc_q15": ("--workload mfcc_q15 --steps 10 --warmup 3", "mfcc_q15_post|cfft_fx_r16_kernel", "mfcc_fixed|cfft_fixed_r16"),
    # the one-launch schedule (variant build MI355X_MFCC_FX_MODE=2): the same bench arguments,
    # run with CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_mfcc1l.so
    "mfcc_q31_onelaunch": ("--workload mfcc_q31 --steps 10 --warmup 3", "cfft_fx_r16_kernel", ""),
    "mfcc_q15_onelaunch": ("--workload mfcc_q15 --steps 10 --warmup 3", "cfft_fx_r16_kernel", ""),
    "mat_mult_f32": ("--workload mat_mult_f32 --steps 6 --warmup 2", "mat_mult_f32_full", ""),
    "mat_mult_q7": ("--workload mat_mult_q7 --steps 10 --warmup 3", "mat_mult_q7_pp", ""),
    "mat_mult_q15": ("--workload mat_mult_q15 --steps 6 --warmup 2", "mat_mult_i8v2", ""),
    "mat_mult_q31": ("--workload mat_mult_q31 --steps 6 --warmup 2", "mat_mult_i8v3", ""),
    "mat_mult_fast_q31": ("--workload mat_mult_fast_q31 --steps 6 --warmup 2", "mat_mult_fast_q31", "mat_mult_fixed"),
}

if __name__ == "__main__":
    print(SPECS[sys.argv[1]][0])
