# Builds the REAL reference scalar path from /root/reference sources into oracle/_ref/.
# Test infrastructure only: the product never links or loads anything built here.
# Flags follow SURVEY.md §8c: the CMake HOST=ON equivalent (__GNUC_PYTHON__ -> scalar
# branches, ARM_MATH_DSP undefined), LOOPUNROLL on (CMake default), no -march, no
# -ffast-math (no FMA contraction on x86-64 baseline).
# Usage:  make -f oracle/ref.mk            (from the repo root)
REF     ?= /root/reference
OUT     ?= oracle/_ref
CC      ?= gcc
CFLAGS  := -O2 -fPIC -D__GNUC_PYTHON__ -DARM_MATH_LOOPUNROLL -ffp-contract=off -w \
           -I$(REF)/Include -I$(REF)/PrivateInclude

T := $(REF)/Source/TransformFunctions
F := $(REF)/Source/FilteringFunctions
M := $(REF)/Source/MatrixFunctions
C := $(REF)/Source/CommonTables
B := $(REF)/Source/BasicMathFunctions
X := $(REF)/Source/ComplexMathFunctions
ST := $(REF)/Source/StatisticsFunctions
FM := $(REF)/Source/FastMathFunctions
SU := $(REF)/Source/SupportFunctions

SRCS := \
  $(T)/arm_cfft_f32.c $(T)/arm_cfft_radix8_f32.c $(T)/arm_cfft_init_f32.c \
  $(T)/arm_cfft_q31.c $(T)/arm_cfft_radix4_q31.c $(T)/arm_cfft_init_q31.c \
  $(T)/arm_cfft_q15.c $(T)/arm_cfft_radix4_q15.c $(T)/arm_cfft_init_q15.c \
  $(T)/arm_bitreversal2.c $(T)/arm_bitreversal.c $(T)/arm_transform_buffer_sizes.c \
  $(T)/arm_rfft_fast_f32.c $(T)/arm_rfft_fast_init_f32.c \
  $(T)/arm_rfft_q31.c $(T)/arm_rfft_init_q31.c $(T)/arm_rfft_q15.c $(T)/arm_rfft_init_q15.c \
  $(B)/arm_shift_q31.c $(B)/arm_shift_q15.c \
  $(F)/arm_fir_f32.c $(F)/arm_fir_init_f32.c $(F)/arm_fir_q15.c $(F)/arm_fir_init_q15.c \
  $(F)/arm_fir_q31.c $(F)/arm_fir_init_q31.c $(F)/arm_fir_fast_q15.c $(F)/arm_fir_fast_q31.c \
  $(F)/arm_conv_f32.c $(F)/arm_conv_q15.c $(F)/arm_conv_q31.c \
  $(F)/arm_conv_fast_q15.c $(F)/arm_conv_fast_q31.c \
  $(F)/arm_conv_partial_f32.c $(F)/arm_conv_partial_q15.c $(F)/arm_conv_partial_q31.c \
  $(F)/arm_conv_partial_fast_q15.c $(F)/arm_conv_partial_fast_q31.c \
  $(F)/arm_correlate_f32.c $(F)/arm_correlate_q15.c $(F)/arm_correlate_q31.c \
  $(F)/arm_correlate_fast_q15.c $(F)/arm_correlate_fast_q31.c \
  $(F)/arm_fir_decimate_f32.c $(F)/arm_fir_decimate_q15.c $(F)/arm_fir_decimate_fast_q15.c \
  $(F)/arm_fir_decimate_q31.c $(F)/arm_fir_decimate_fast_q31.c \
  $(F)/arm_fir_decimate_init_f32.c $(F)/arm_fir_decimate_init_q15.c $(F)/arm_fir_decimate_init_q31.c \
  $(F)/arm_fir_interpolate_f32.c $(F)/arm_fir_interpolate_q15.c $(F)/arm_fir_interpolate_q31.c \
  $(F)/arm_fir_interpolate_init_f32.c $(F)/arm_fir_interpolate_init_q15.c $(F)/arm_fir_interpolate_init_q31.c \
  $(F)/arm_fir_sparse_f32.c $(F)/arm_fir_sparse_q31.c $(F)/arm_fir_sparse_q15.c $(F)/arm_fir_sparse_q7.c \
  $(F)/arm_fir_sparse_init_f32.c $(F)/arm_fir_sparse_init_q31.c $(F)/arm_fir_sparse_init_q15.c \
  $(F)/arm_fir_sparse_init_q7.c \
  $(F)/arm_fir_lattice_f32.c $(F)/arm_fir_lattice_q31.c $(F)/arm_fir_lattice_q15.c \
  $(F)/arm_fir_lattice_init_f32.c $(F)/arm_fir_lattice_init_q31.c $(F)/arm_fir_lattice_init_q15.c \
  $(F)/arm_conv_opt_q15.c $(F)/arm_conv_opt_q7.c $(F)/arm_conv_fast_opt_q15.c \
  $(F)/arm_conv_partial_opt_q15.c $(F)/arm_conv_partial_opt_q7.c $(F)/arm_conv_partial_fast_opt_q15.c \
  $(F)/arm_correlate_opt_q15.c $(F)/arm_correlate_opt_q7.c $(F)/arm_correlate_fast_opt_q15.c \
  $(SU)/arm_copy_q15.c $(SU)/arm_fill_q15.c \
  $(F)/arm_fir_q7.c $(F)/arm_fir_init_q7.c $(F)/arm_conv_q7.c $(F)/arm_conv_partial_q7.c $(F)/arm_correlate_q7.c \
  $(M)/arm_mat_mult_f32.c $(M)/arm_mat_init_f32.c $(M)/arm_mat_vec_mult_f32.c \
  $(M)/arm_mat_mult_q7.c $(M)/arm_mat_mult_q15.c $(M)/arm_mat_mult_q31.c $(M)/arm_mat_mult_opt_q31.c $(M)/arm_mat_mult_fast_q15.c $(M)/arm_mat_mult_fast_q31.c $(M)/arm_mat_init_q7.c $(M)/arm_mat_init_q15.c $(M)/arm_mat_init_q31.c \
  $(T)/arm_mfcc_f32.c $(T)/arm_mfcc_init_f32.c $(ST)/arm_absmax_f32.c $(B)/arm_scale_f32.c \
  $(B)/arm_mult_f32.c $(B)/arm_dot_prod_f32.c $(B)/arm_offset_f32.c $(X)/arm_cmplx_mag_f32.c \
  $(FM)/arm_vlog_f32.c \
  $(T)/arm_mfcc_q31.c $(T)/arm_mfcc_init_q31.c $(ST)/arm_absmax_q31.c $(FM)/arm_divide_q31.c \
  $(B)/arm_scale_q31.c $(B)/arm_mult_q31.c $(B)/arm_abs_q31.c $(X)/arm_cmplx_mag_q31.c $(FM)/arm_sqrt_q31.c \
  $(B)/arm_dot_prod_q31.c $(FM)/arm_vlog_q31.c $(B)/arm_offset_q31.c $(M)/arm_mat_vec_mult_q31.c \
  $(T)/arm_mfcc_q15.c $(T)/arm_mfcc_init_q15.c $(ST)/arm_absmax_q15.c $(FM)/arm_divide_q15.c \
  $(B)/arm_scale_q15.c $(B)/arm_mult_q15.c $(B)/arm_abs_q15.c $(X)/arm_cmplx_mag_q15.c $(B)/arm_dot_prod_q15.c \
  $(M)/arm_mat_vec_mult_q15.c \
  $(C)/arm_common_tables.c $(C)/arm_const_structs.c

OBJS := $(patsubst $(REF)/Source/%.c,$(OUT)/obj/%.o,$(SRCS))

all: $(OUT)/libcmsisdsp_ref.so $(OUT)/bench_ref

$(OUT)/obj/%.o: $(REF)/Source/%.c
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/libcmsisdsp_ref.so: $(OBJS)
	$(CC) -shared -Wl,-Bsymbolic -o $@ $(OBJS) -lm

# Timing driver (CPU baseline kind "reference"): our own source, linked to the reference objects.
$(OUT)/bench_ref: oracle/bench_cpu.c $(OBJS)
	$(CC) -O2 -D__GNUC_PYTHON__ -DARM_MATH_LOOPUNROLL -I$(REF)/Include -I$(REF)/PrivateInclude \
	  -DBENCH_AGAINST_REFERENCE -o $@ oracle/bench_cpu.c $(OBJS) -lm -lpthread

clean:
	rm -rf $(OUT)/obj $(OUT)/libcmsisdsp_ref.so $(OUT)/bench_ref
.PHONY: all clean
