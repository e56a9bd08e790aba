# oracle/enc.mk — builds the REFERENCE ENCODER itself (every C source of Source/Lib/Common, Source/Lib/Encoder and
# third_party/fastfeat, straight from /root/reference with gcc) into oracle/_ref/enc/libsvtenc.so, and the drop-in
# harness that links it with libsvtgpu (oracle/ref_harness/enc_drop_in.c; tests/test_encoder_drop_in.py).
# Test infrastructure only: the encoder's public API drives its own DLF / CDEF / LR process
# bodies with libsvtgpu installed.  The reference's cmake build is NOT used.
#
# C-only configuration (the reference's COMPILE_C_ONLY: no ARCH_X86_64, so its NASM sources -- which this image cannot
# assemble -- are not needed and the RTCD setup binds the C kernels).  One generated file: EbVersion.h, which the
# reference's cmake instantiates from its own template Source/Lib/Common/Codec/EbVersion.h.in (configure_file,
# Source/Lib/Common/Codec/CMakeLists.txt:15-17) with the project version of CMakeLists.txt:14 (2.1.0); the recipe
# does the same substitution with sed, into the build directory.
#
#   make -f oracle/enc.mk -j8            # from the repo root
REF      ?= /root/reference
OUT      ?= oracle/_ref/enc
S        := $(REF)/Source
CC       ?= gcc
SVTGPU   := svt-av1_pro-anchor-v2.1.0-_amd/lib
INC      := -I$(S)/API -I$(S)/Lib/Common/Codec -I$(S)/Lib/Common/C_DEFAULT -I$(S)/Lib/Encoder/Codec \
            -I$(S)/Lib/Encoder/C_DEFAULT -I$(S)/Lib/Encoder/Globals -I$(REF)/third_party/fastfeat -I$(REF) -I$(OUT)/gen
CFLAGS   := -O2 -fPIC -w -std=gnu99 $(INC)
ENC_SRC  := $(wildcard $(S)/Lib/Common/Codec/*.c $(S)/Lib/Common/C_DEFAULT/*.c $(S)/Lib/Encoder/Codec/*.c \
                       $(S)/Lib/Encoder/C_DEFAULT/*.c $(S)/Lib/Encoder/Globals/*.c $(REF)/third_party/fastfeat/*.c)
ENC_OBJ  := $(patsubst $(REF)/%.c,$(OUT)/obj/%.o,$(ENC_SRC))

all: $(OUT)/libsvtenc.so $(OUT)/enc_drop_in $(OUT)/nss/enc_drop_in $(OUT)/ccso/enc_drop_in

$(OUT)/gen/EbVersion.h: $(S)/Lib/Common/Codec/EbVersion.h.in
	@mkdir -p $(dir $@)
	sed 's/@PACKAGE_VERSION_STRING@/v2.1.0/' $< > $@

$(OUT)/obj/%.o: $(REF)/%.c $(OUT)/gen/EbVersion.h
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/libsvtenc.so: $(ENC_OBJ)
	$(CC) -shared -o $@ $^ -lm -lpthread

# the harness: the reference's public API + include/svtgpu_rtcd.h (no casts: the install compiles against the
# reference's own RTCD declarations), the frame-level hooks (enc_frame_hooks.c) defined in the executable
$(OUT)/enc_drop_in: oracle/ref_harness/enc_drop_in.c oracle/ref_harness/enc_frame_hooks.c $(OUT)/libsvtenc.so \
                    $(SVTGPU)/libsvtgpu.so
	$(CC) -O2 -w -std=gnu99 $(INC) -Iinclude -Werror=incompatible-pointer-types $(filter %.c,$^) -o $@ \
	    -L$(OUT) -lsvtenc -L$(SVTGPU) -lsvtgpu -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../$(SVTGPU)' \
	    -rdynamic -ldl -lm -lpthread

# The same encoder with the CDEF process body's per-segment CPU search removed (INTEGRATION.md §2 applied): a /tmp copy
# of EbCdefProcess.c edited by oracle/ref_harness/no_seg_search.py (one call statement), compiled into
# $(OUT)/nss/libsvtenc.so beside the unchanged objects, and the harness linked against it (frame mode only: the hooked
# finish_cdef_search searches the frame on the device; the encoder's own finish_cdef_search would find no tables).
NSS_TMP  ?= /tmp/svtgpu_enc_nss
$(NSS_TMP)/EbCdefProcess.c: $(S)/Lib/Encoder/Codec/EbCdefProcess.c oracle/ref_harness/no_seg_search.py
	@mkdir -p $(dir $@)
	python3 oracle/ref_harness/no_seg_search.py $< $@

$(OUT)/nss/EbCdefProcess.o: $(NSS_TMP)/EbCdefProcess.c $(OUT)/gen/EbVersion.h
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/nss/libsvtenc.so: $(filter-out %/EbCdefProcess.o,$(ENC_OBJ)) $(OUT)/nss/EbCdefProcess.o
	$(CC) -shared -o $@ $^ -lm -lpthread

$(OUT)/nss/enc_drop_in: oracle/ref_harness/enc_drop_in.c oracle/ref_harness/enc_frame_hooks.c $(OUT)/nss/libsvtenc.so \
                        $(SVTGPU)/libsvtgpu.so
	$(CC) -O2 -w -std=gnu99 $(INC) -Iinclude -Werror=incompatible-pointer-types $(filter %.c,$^) -o $@ \
	    -L$(OUT)/nss -lsvtenc -L$(SVTGPU) -lsvtgpu -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../../$(SVTGPU)' \
	    -rdynamic -ldl -lm -lpthread

# The encoder with the fork's CCSO switched back on: a /tmp copy of EbCdefProcess.c with the two
# commented calls (ccso_search / ccso_frame, :621-623) uncommented by oracle/ref_harness/with_ccso.py, compiled into
# $(OUT)/ccso/libsvtenc.so; its harness runs the CPU CCSO (cpu mode) or, through the hooks, the device's (frame mode).
CCSO_TMP ?= /tmp/svtgpu_enc_ccso
$(CCSO_TMP)/EbCdefProcess.c: $(S)/Lib/Encoder/Codec/EbCdefProcess.c oracle/ref_harness/with_ccso.py
	@mkdir -p $(dir $@)
	python3 oracle/ref_harness/with_ccso.py $< $@

$(OUT)/ccso/EbCdefProcess.o: $(CCSO_TMP)/EbCdefProcess.c $(OUT)/gen/EbVersion.h
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/ccso/libsvtenc.so: $(filter-out %/EbCdefProcess.o,$(ENC_OBJ)) $(OUT)/ccso/EbCdefProcess.o
	$(CC) -shared -o $@ $^ -lm -lpthread

$(OUT)/ccso/enc_drop_in: oracle/ref_harness/enc_drop_in.c oracle/ref_harness/enc_frame_hooks.c $(OUT)/ccso/libsvtenc.so \
                         $(SVTGPU)/libsvtgpu.so
	$(CC) -O2 -w -std=gnu99 $(INC) -Iinclude -Werror=incompatible-pointer-types $(filter %.c,$^) -o $@ \
	    -L$(OUT)/ccso -lsvtenc -L$(SVTGPU) -lsvtgpu -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../../$(SVTGPU)' \
	    -rdynamic -ldl -lm -lpthread

clean:
	rm -rf $(OUT)
.PHONY: all clean
