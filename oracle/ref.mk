# Builds the REFERENCE (BioinformaticsArchive/HSA) from its own sources where
# they lie under /root/reference, into oracle/_ref/ only.  Test infrastructure:
# the outputs are the oracle's pin (golden vectors) and the optional CPU baseline;
# nothing under oracle/ is linked into the product library.
#
# Flags = reference Makefile:3 minus -static, plus -fgnu89-inline (SURVEY §4.3:
# without it gcc 11 fails to link bwt_array.c's C99 inline definitions) and -fPIC.
REF      ?= /root/reference
OUT      ?= $(CURDIR)/_ref
CC       ?= gcc
REFFLAGS  = -w -g -O3 -funroll-loops -march=nocona -maccumulate-outgoing-args \
            -fno-stack-protector -msse3 -fgnu89-inline -fPIC
REFOBJS   = bwtaln bwtgap BWT BWTConstruct utils dictionary DNACount HSP iniparser \
            inistrlib MemManager MiscUtilities QSufSort 2BWT-Builder TextConverter Timing \
            bamlite 2BWT-Interface bwaseqio r250 cs2nt bwtse kstring stdaln bwt_array
OBJS      = $(addprefix $(OUT)/obj/,$(addsuffix .o,$(REFOBJS)))

all: $(OUT)/HSA $(OUT)/ref_probe $(OUT)/ref_mgcap $(OUT)/ref_extcap $(OUT)/HSA_gpu $(OUT)/HSA_gpu_mg $(OUT)/HSA_gpu_all \
     $(OUT)/ref_probe_gpu $(OUT)/HSA_sam

$(OUT)/obj/%.o: $(REF)/%.c
	@mkdir -p $(OUT)/obj
	$(CC) -c $(REFFLAGS) -I$(REF) $< -o $@

$(OUT)/libhsaref.a: $(OBJS)
	rm -f $@ && ar rcs $@ $(OBJS)

$(OUT)/HSA: $(OUT)/obj/main.o $(OUT)/libhsaref.a
	$(CC) $(REFFLAGS) $^ -lm -lz -o $@

# ref_probe.c is ours; it drives the reference's bwa_cal_sa_reg_gap batch by batch
# and records which reads reached bwt_splice_match via --wrap.
$(OUT)/ref_probe: ref_probe.c $(OUT)/libhsaref.a
	$(CC) $(REFFLAGS) -I$(REF) ref_probe.c $(OUT)/libhsaref.a \
	    -Wl,--wrap=bwt_splice_match -lm -lz -o $@

# HSA_gpu: the reference's own HSA binary with OUR bwa_cal_sa_reg_gap linked in
# (INTEGRATION.md).  The reference definition is weakened in a copy of bwtaln.o
# (verified there), our strong definition comes from bwtaln_gpu.o, and
# the search core from libhsa_gpu.so.  Only built when the product library exists;
# the drop-in test (tests/test_gpu_dropin.py) compares its SAM with the reference's.
GPULIB    = $(CURDIR)/../hsa_amd/libhsa_gpu.so
GPUOBJ    = $(CURDIR)/../hsa_amd/csrc/bwtaln_gpu.o
WEAKOBJS  = $(filter-out $(OUT)/obj/bwtaln.o,$(OBJS)) $(OUT)/obj/bwtaln_weak.o

$(OUT)/obj/bwtaln_weak.o: $(OUT)/obj/bwtaln.o
	objcopy --weaken-symbol=bwa_cal_sa_reg_gap $< $@

$(OUT)/HSA_gpu: $(OUT)/obj/main.o $(WEAKOBJS) $(GPUOBJ) $(GPULIB)
	$(CC) $(REFFLAGS) $(OUT)/obj/main.o $(WEAKOBJS) $(GPUOBJ) -L$(dir $(GPULIB)) -lhsa_gpu \
	    -Wl,-rpath,'$$ORIGIN/../../hsa_amd' -lm -lz -lpthread -o $@

# ref_mgcap.c is ours: it records every bwt_match_gap call (inputs, widths before and
# after, hits).  bwtgap.o enters twice: weakened, so that every call -- including
# bwt_splice_match's own, which go through the PLT under -fPIC -- reaches the
# recorder; and renamed (ref_bwt_match_gap) with every other global made local, the
# unmodified reference function the recorder calls.
$(OUT)/obj/bwtgap_weak.o: $(OUT)/obj/bwtgap.o
	objcopy --weaken-symbol=bwt_match_gap $< $@

$(OUT)/obj/bwtgap_ren.o: $(OUT)/obj/bwtgap.o
	objcopy --redefine-sym bwt_match_gap=ref_bwt_match_gap $< $@.tmp
	objcopy --keep-global-symbol=ref_bwt_match_gap $@.tmp $@
	rm -f $@.tmp

CAPOBJS   = $(filter-out $(OUT)/obj/bwtgap.o,$(OBJS)) $(OUT)/obj/bwtgap_weak.o $(OUT)/obj/bwtgap_ren.o

$(OUT)/ref_mgcap: ref_mgcap.c $(CAPOBJS)
	$(CC) $(REFFLAGS) -I$(REF) ref_mgcap.c $(CAPOBJS) -lm -lz -o $@

# ref_extcap.c is ours: it records every seed extension of the splice path
# (bwt_extend_foreward / bwt_extend_backward, bwtgap.c:640-663), the same way.
$(OUT)/obj/bwtgap_weakx.o: $(OUT)/obj/bwtgap.o
	objcopy --weaken-symbol=bwt_extend_foreward --weaken-symbol=bwt_extend_backward $< $@

$(OUT)/obj/bwtgap_renx.o: $(OUT)/obj/bwtgap.o
	objcopy --redefine-sym bwt_extend_foreward=ref_bwt_extend_foreward \
	        --redefine-sym bwt_extend_backward=ref_bwt_extend_backward $< $@.tmp
	objcopy --keep-global-symbol=ref_bwt_extend_foreward --keep-global-symbol=ref_bwt_extend_backward $@.tmp $@
	rm -f $@.tmp

EXTOBJS   = $(filter-out $(OUT)/obj/bwtgap.o,$(OBJS)) $(OUT)/obj/bwtgap_weakx.o $(OUT)/obj/bwtgap_renx.o

$(OUT)/ref_extcap: ref_extcap.c $(EXTOBJS)
	$(CC) $(REFFLAGS) -I$(REF) ref_extcap.c $(EXTOBJS) -lm -lz -o $@

# HSA_gpu_mg: as HSA_gpu, with bwt_match_gap weakened too, so the host's splice path
# (bwt_splice_match, bwtgap.c:748) calls OUR bwt_match_gap for its seed and anchor
# searches (bwtgap.c:812, :919, :1192).
MGOBJS    = $(filter-out $(OUT)/obj/bwtaln.o $(OUT)/obj/bwtgap.o,$(OBJS)) $(OUT)/obj/bwtaln_weak.o \
            $(OUT)/obj/bwtgap_weak.o

GPUOBJ_MG = $(CURDIR)/../hsa_amd/csrc/bwtgap_gpu.o

$(OUT)/HSA_gpu_mg: $(OUT)/obj/main.o $(MGOBJS) $(GPUOBJ) $(GPUOBJ_MG) $(GPULIB)
	$(CC) $(REFFLAGS) $(OUT)/obj/main.o $(MGOBJS) $(GPUOBJ) $(GPUOBJ_MG) -L$(dir $(GPULIB)) -lhsa_gpu \
	    -Wl,-rpath,'$$ORIGIN/../../hsa_amd' -lm -lz -lpthread -o $@

# HSA_gpu_all: every drop-in entry point replaced -- bwa_cal_sa_reg_gap, bwt_match_gap
# (as HSA_gpu_mg), the splice path's seed extensions bwt_extend_backward /
# bwt_extend_foreward (weakened in bwtgap.o too: hsa_amd/csrc/bwtext_gpu.c runs the
# splice path of a batch's fallback reads as coroutines and their extensions as GPU
# batches), bwt_cal_width (weakened in bwtaln.o: the splice path's widths from a table
# filled on the GPU, bwtext_gpu.c), the splice path's SA -> position lookups (bwtgap.o's
# reference to BWTRetrievePositionFromSAIndex renamed to hsa_splice_sa_position, so the
# SAM stage keeps the host's own), and the SAM stage's bwa_cal_pac_pos, weakened in bwtse.o, so that
# generate_sam_se_core (bwtse.c:911) calls OUR bwa_cal_pac_pos (hsa_amd/csrc/bwtse_gpu.c:
# the batch's SA -> position lookups on the GPU) -- and generate_sam_se_core itself, weakened
# in bwtse.o too: hsa_amd/csrc/bwtsam_gpu.c runs the SAM stage on host threads.
$(OUT)/obj/bwtse_weak.o: $(OUT)/obj/bwtse.o
	objcopy --weaken-symbol=bwa_cal_pac_pos --weaken-symbol=generate_sam_se_core $< $@

$(OUT)/obj/bwtaln_weak_all.o: $(OUT)/obj/bwtaln.o
	objcopy --weaken-symbol=bwa_cal_sa_reg_gap --weaken-symbol=bwt_cal_width $< $@

$(OUT)/obj/bwtgap_weak_all.o: $(OUT)/obj/bwtgap.o
	objcopy --weaken-symbol=bwt_match_gap --weaken-symbol=bwt_extend_foreward \
	        --weaken-symbol=bwt_extend_backward \
	        --redefine-sym BWTRetrievePositionFromSAIndex=hsa_splice_sa_position $< $@

ALLOBJS   = $(filter-out $(OUT)/obj/bwtaln.o $(OUT)/obj/bwtgap.o $(OUT)/obj/bwtse.o,$(OBJS)) \
            $(OUT)/obj/bwtaln_weak_all.o $(OUT)/obj/bwtgap_weak_all.o $(OUT)/obj/bwtse_weak.o
GPUOBJ_SA = $(CURDIR)/../hsa_amd/csrc/bwtse_gpu.o $(CURDIR)/../hsa_amd/csrc/bwtsam_gpu.o
GPUOBJ_EX = $(CURDIR)/../hsa_amd/csrc/bwtext_gpu.o

$(OUT)/HSA_gpu_all: $(OUT)/obj/main.o $(ALLOBJS) $(GPUOBJ) $(GPUOBJ_MG) $(GPUOBJ_SA) $(GPUOBJ_EX) $(GPULIB)
	$(CC) $(REFFLAGS) $(OUT)/obj/main.o $(ALLOBJS) $(GPUOBJ) $(GPUOBJ_MG) $(GPUOBJ_SA) $(GPUOBJ_EX) \
	    -L$(dir $(GPULIB)) -lhsa_gpu -Wl,-rpath,'$$ORIGIN/../../hsa_amd' -lm -lz -lpthread -o $@

# ref_probe_gpu: ref_probe.c linked as HSA_gpu_all (every drop-in entry point ours, the
# reference's bwt_splice_match in between): bench.py times the drop-in end to end on
# bwa_seq_t batches with it and compares its hits with ref_probe's, read for read.
$(OUT)/ref_probe_gpu: ref_probe.c $(ALLOBJS) $(GPUOBJ) $(GPUOBJ_MG) $(GPUOBJ_SA) $(GPUOBJ_EX) $(GPULIB)
	$(CC) $(REFFLAGS) -DHSA_GPU_PROBE -I$(REF) ref_probe.c $(ALLOBJS) $(GPUOBJ) $(GPUOBJ_MG) $(GPUOBJ_SA) \
	    $(GPUOBJ_EX) -L$(dir $(GPULIB)) -lhsa_gpu -Wl,-rpath,'$$ORIGIN/../../hsa_amd' -lm -lz -lpthread -o $@

# HSA_sam: the reference's HSA (CPU, its own search and SA -> position) with only the SAM
# stage replaced: generate_sam_se_core weakened in bwtse.o, hsa_amd/csrc/bwtsam_gpu.c's on
# host threads (no GPU).  tests/test_sam_cpu.py compares its SAM with the reference's.
$(OUT)/obj/bwtse_weak_sam.o: $(OUT)/obj/bwtse.o
	objcopy --weaken-symbol=generate_sam_se_core $< $@

# ... and with bwa_print_sam1 weakened as well (the printing guard's test supplies a host
# function that prints other bytes)
$(OUT)/obj/bwtse_weak_sam_print.o: $(OUT)/obj/bwtse.o
	objcopy --weaken-symbol=generate_sam_se_core --weaken-symbol=bwa_print_sam1 $< $@

SAMOBJS   = $(filter-out $(OUT)/obj/bwtse.o,$(OBJS)) $(OUT)/obj/bwtse_weak_sam.o
GPUOBJ_SAM = $(CURDIR)/../hsa_amd/csrc/bwtsam_gpu.o

$(OUT)/HSA_sam: $(OUT)/obj/main.o $(SAMOBJS) $(GPUOBJ_SAM) $(OUT)/obj/bwtse_weak_sam_print.o
	$(CC) $(REFFLAGS) $(OUT)/obj/main.o $(SAMOBJS) $(GPUOBJ_SAM) -lm -lz -lpthread -o $@

clean:
	rm -rf $(OUT)

.PHONY: all clean
