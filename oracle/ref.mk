# oracle/ref.mk — builds the REFERENCE's own C (and AVX2) hot-path sources, straight from
# /root/reference with gcc, into oracle/_ref/ (git-ignored, shipped to the GPU box by gpurun).
# Test infrastructure only: the golden-vector generators and the reference CPU baseline.
# The reference's cmake build system is NOT used; only its source files are compiled directly.
#
#   make -f oracle/ref.mk            # from the repo root
REF      ?= /root/reference
OUT      ?= oracle/_ref
S        := $(REF)/Source
CC       ?= gcc
INC      := -I$(S)/API -I$(S)/Lib/Common/Codec -I$(S)/Lib/Common/C_DEFAULT -I$(S)/Lib/Encoder/Codec \
            -I$(S)/Lib/Encoder/C_DEFAULT -I$(S)/Lib/Encoder/Globals -I$(S)/Lib/Common/ASM_AVX2 \
            -I$(S)/Lib/Encoder/ASM_AVX2 -I$(S)/Lib/Common/ASM_SSE2 -I$(S)/Lib/Common/ASM_SSE4_1 \
            -I$(REF)/third_party/aom/inc -I$(REF)/third_party/cpuinfo/include -I$(REF) -Ioracle/ref_harness
CFLAGS   := -O2 -fPIC -ffunction-sections -fdata-sections -DARCH_X86_64=1 -w $(INC)

# reference C sources (semantic definitions of the kernels)
REF_C    := Lib/Common/Codec/EbCdef.c Lib/Encoder/Codec/EbEncCdef.c Lib/Common/Codec/common_dsp_rtcd.c \
            Lib/Encoder/Codec/aom_dsp_rtcd.c Lib/Common/Codec/EbUtility.c
DLF_C    := Lib/Common/Codec/EbDeblockingCommon.c Lib/Encoder/Codec/EbDeblockingFilter.c
LR_C     := Lib/Common/Codec/convolve.c Lib/Common/Codec/EbRestoration.c Lib/Common/Codec/EbPictureBufferDesc.c \
            Lib/Common/Codec/EbMalloc.c Lib/Common/Codec/EbLog.c Lib/Common/Codec/EbSuperRes.c Lib/Common/C_DEFAULT/EbPictureOperators_C.c \
            Lib/Common/Codec/EbThreads.c Lib/Common/Codec/EbBlockStructures.c \
            Lib/Common/Codec/EbPictureOperators.c Lib/Encoder/Codec/EbRestorationPick.c Lib/Encoder/Codec/EbEntropyCoding.c
MD_C     := Lib/Encoder/C_DEFAULT/EbComputeSAD_C.c Lib/Encoder/C_DEFAULT/variance.c Lib/Encoder/Codec/EbPsnr.c \
            Lib/Encoder/Codec/EbEncInterPrediction.c Lib/Common/C_DEFAULT/EbPictureOperators_C.c \
            Lib/Common/Codec/EbPictureOperators.c
# frame-level drivers the pipeline generator reaches: get_recon_pic (EbRestProcess.c), the lambda table
# (EbModeDecisionProcess.c), svt_aom_compute_rd_mult (EbRateControlProcess.c), the quantizer tables (EbInvTransforms.c)
PIPE_C   := Lib/Encoder/Codec/EbRestProcess.c Lib/Encoder/Codec/EbModeDecisionProcess.c \
            Lib/Encoder/Codec/EbRateControlProcess.c Lib/Common/Codec/EbInvTransforms.c
# reference AVX2 sources (the CPU baseline the north star names)
REF_AVX2 := Lib/Common/ASM_AVX2/cdef_block_avx2.c Lib/Encoder/ASM_AVX2/EbCdef_AVX2.c
# ... and the rest of the AVX2 / SSE2 kernels an AVX2 host binds for the bench's stages (ref_bench)
BENCH_SIMD := Lib/Common/ASM_AVX2/selfguided_avx2.c Lib/Common/ASM_AVX2/wiener_convolve_avx2.c \
            Lib/Common/ASM_AVX2/highbd_convolve_avx2.c Lib/Encoder/ASM_AVX2/pickrst_avx2.c \
            Lib/Encoder/ASM_AVX2/EbComputeSAD_Intrinsic_AVX2.c \
            Lib/Encoder/ASM_AVX2/variance_avx2.c Lib/Encoder/ASM_AVX2/variance_impl_avx2.c \
            Lib/Encoder/ASM_AVX2/highbd_variance_avx2.c Lib/Encoder/ASM_AVX2/sse_avx2.c \
            Lib/Common/ASM_AVX2/EbPictureOperators_Intrinsic_AVX2.c Lib/Common/ASM_SSE2/EbDeblockingFilter_Intrinsic_SSE2.c \
            Lib/Common/ASM_SSE2/EbPictureOperators_Intrinsic_SSE2.c

C_OBJ    := $(patsubst %.c,$(OUT)/obj/%.o,$(REF_C))
DLF_OBJ  := $(patsubst %.c,$(OUT)/obj/%.o,$(DLF_C))
MD_OBJ   := $(patsubst %.c,$(OUT)/obj/%.o,$(MD_C))
LR_OBJ   := $(patsubst %.c,$(OUT)/obj/%.o,$(LR_C))
AVX2_OBJ := $(patsubst %.c,$(OUT)/obj/%.o,$(REF_AVX2))
SIMD_OBJ := $(patsubst %.c,$(OUT)/obj/%.o,$(BENCH_SIMD))
PIPE_OBJ := $(patsubst %.c,$(OUT)/obj/%.o,$(PIPE_C))

all: $(OUT)/gen_golden_cdef $(OUT)/gen_golden_dlf $(OUT)/gen_golden_md $(OUT)/gen_golden_lr $(OUT)/gen_golden_pipe \
     $(OUT)/gen_golden_shims $(OUT)/rtcd_pipe $(OUT)/ref_bench $(OUT)/gen_golden_me $(OUT)/gen_golden_frame \
     $(OUT)/rtcd_install $(OUT)/gen_golden_ccso

$(OUT)/obj/Lib/Common/ASM_AVX2/%.o $(OUT)/obj/Lib/Encoder/ASM_AVX2/%.o: CFLAGS += -mavx2
$(OUT)/obj/Lib/Common/ASM_SSE2/%.o: CFLAGS += -msse2
# RunEmms (x86 `emms`, only reachable through aom_clear_system_state) lives in NASM sources this image cannot
# assemble; the generic (non-x86) configuration of this file skips that call and computes the same values.
$(OUT)/obj/Lib/Encoder/Codec/EbRestorationPick.o: CFLAGS += -UARCH_X86_64
$(OUT)/obj/%.o: $(S)/%.c
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/gen_golden_cdef: oracle/ref_harness/gen_golden_cdef.c $(C_OBJ)
	$(CC) $(CFLAGS) $^ -o $@ -Wl,--gc-sections -lm

$(OUT)/gen_golden_dlf: oracle/ref_harness/gen_golden_dlf.c $(DLF_OBJ) $(C_OBJ)
	$(CC) $(CFLAGS) $^ -o $@ -Wl,--gc-sections -lm

$(OUT)/gen_golden_md: oracle/ref_harness/gen_golden_md.c $(MD_OBJ) $(C_OBJ)
	$(CC) $(CFLAGS) $^ -o $@ -Wl,--gc-sections -lm

$(OUT)/gen_golden_lr: oracle/ref_harness/gen_golden_lr.c $(sort $(LR_OBJ) $(MD_OBJ) $(C_OBJ))
	$(CC) $(CFLAGS) $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -lm -lpthread

# whole-frame DLF -> CDEF -> LR through the reference's own frame-level code; the two harness units compile the
# reference's EbCdefProcess.c / EncModeConfig.c (static functions) as they lie
$(OUT)/gen_golden_pipe: oracle/ref_harness/gen_golden_pipe.c oracle/ref_harness/ref_cdef_process.c \
                        oracle/ref_harness/ref_mode_config.c $(sort $(LR_OBJ) $(MD_OBJ) $(DLF_OBJ) $(C_OBJ) $(PIPE_OBJ))
	$(CC) $(CFLAGS) $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -lm -lpthread

# the same frame code with the reference's RTCD pointers bound to libsvtgpu's shims (no casts: the compile fails on
# any prototype mismatch); run on the GPU box by tests/test_rtcd_bind.py
SVTGPU_SO := svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so
$(OUT)/rtcd_pipe: oracle/ref_harness/gen_golden_pipe.c oracle/ref_harness/ref_cdef_process.c \
                  oracle/ref_harness/ref_mode_config.c $(sort $(LR_OBJ) $(MD_OBJ) $(DLF_OBJ) $(C_OBJ) $(PIPE_OBJ)) $(SVTGPU_SO)
	@mkdir -p $(OUT)/obj/bind
	$(CC) $(filter-out -w,$(CFLAGS)) -DSVTGPU_BIND -Iinclude -Werror=incompatible-pointer-types -Werror=discarded-qualifiers \
	    -c oracle/ref_harness/gen_golden_pipe.c -o $(OUT)/obj/bind/gen_golden_pipe.o
	$(CC) $(CFLAGS) $(OUT)/obj/bind/gen_golden_pipe.o $(filter-out %gen_golden_pipe.c,$(filter %.c,$^)) $(filter %.o,$^) \
	    -o $@ -Wl,--gc-sections -L$(dir $(SVTGPU_SO)) -lsvtgpu -Wl,-rpath,'$$ORIGIN/../../$(dir $(SVTGPU_SO))' -lm -lpthread

# the install point of the RTCD shims against the reference's own init_fn_ptr (av1me.c): pointer comparisons only,
# no device call (tests/test_rtcd_bind.py, CPU)
$(OUT)/rtcd_install: oracle/ref_harness/rtcd_install.c $(OUT)/obj/Lib/Encoder/Codec/av1me.o $(sort $(MD_OBJ) $(C_OBJ)) \
                     $(SVTGPU_SO)
	$(CC) $(filter-out -w,$(CFLAGS)) -Iinclude -Werror=incompatible-pointer-types -Werror=discarded-qualifiers \
	    $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -L$(dir $(SVTGPU_SO)) -lsvtgpu \
	    -Wl,-rpath,'$$ORIGIN/../../$(dir $(SVTGPU_SO))' -ldl -lm -lpthread

# compile-only check of every shim prototype against the reference's pointer types (tests/test_rtcd_bind.py, CPU)
bindcheck:
	$(CC) $(filter-out -w,$(CFLAGS)) -DSVTGPU_BIND -Iinclude -Werror=incompatible-pointer-types \
	    -Werror=discarded-qualifiers -fsyntax-only oracle/ref_harness/gen_golden_pipe.c
.PHONY: bindcheck

# the round-2 RTCD shims (C, and the AVX2-only svt_cdef_filter_block_8xn_16)
$(OUT)/gen_golden_shims: oracle/ref_harness/gen_golden_shims.c $(sort $(LR_OBJ) $(MD_OBJ) $(C_OBJ)) $(AVX2_OBJ)
	$(CC) $(CFLAGS) $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -lm -lpthread

# the reference's CPU path on the bench workload (bench.py cpu_baseline, kind "reference")
$(OUT)/ref_bench: oracle/ref_harness/ref_bench.c $(sort $(LR_OBJ) $(MD_OBJ) $(DLF_OBJ) $(C_OBJ)) $(AVX2_OBJ) $(SIMD_OBJ)
	$(CC) $(CFLAGS) $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -lm -lpthread

clean:
	rm -rf $(OUT)
.PHONY: all clean

# open-loop ME SAD: the reference's EbMotionEstimation.c kernels + svt_sad_loop_kernel_c
ME_C     := Lib/Encoder/Codec/EbMotionEstimation.c Lib/Encoder/Codec/EbProductCodingLoop.c Lib/Encoder/Codec/mcomp.c \
            Lib/Encoder/Codec/EbRateDistortionCost.c
ME_OBJ   := $(patsubst %.c,$(OUT)/obj/%.o,$(ME_C))
$(OUT)/gen_golden_me: oracle/ref_harness/gen_golden_me.c $(sort $(ME_OBJ) $(MD_OBJ) $(C_OBJ))
	$(CC) $(CFLAGS) $^ -o $@ -Wl,--gc-sections -lm -lpthread

# frame-buffer work around the path: conversions, reference padding, frame extension
FRAME_C  := Lib/Common/C_DEFAULT/EbPackUnPack_C.c Lib/Common/Codec/EbMcp.c
FRAME_OBJ := $(patsubst %.c,$(OUT)/obj/%.o,$(FRAME_C))
$(OUT)/gen_golden_frame: oracle/ref_harness/gen_golden_frame.c $(sort $(FRAME_OBJ) $(LR_OBJ) $(MD_OBJ) $(C_OBJ))
	$(CC) $(CFLAGS) $^ -o $@ -Wl,--gc-sections -lm -lpthread

# CCSO: the fork's EbCcso.c / EbPickccso.c; ccso_search reaches svt_aom_get_recon_pic (EbRestProcess.c),
# svt_av1_setup_dst_planes (EbDeblockingFilter.c) and svt_aom_get_syntax_rate_from_cdf (EbMdRateEstimation.c)
CCSO_C   := Lib/Common/Codec/EbCcso.c Lib/Encoder/Codec/EbPickccso.c Lib/Encoder/Codec/EbMdRateEstimation.c
CCSO_OBJ := $(patsubst %.c,$(OUT)/obj/%.o,$(CCSO_C)) $(OUT)/obj/Lib/Common/ASM_AVX2/ccso_avx2.o
$(OUT)/gen_golden_ccso: oracle/ref_harness/gen_golden_ccso.c $(sort $(CCSO_OBJ) $(LR_OBJ) $(MD_OBJ) $(DLF_OBJ) $(C_OBJ) $(PIPE_OBJ))
	$(CC) $(CFLAGS) $(filter %.c,$^) $(filter %.o,$^) -o $@ -Wl,--gc-sections -lm -lpthread
