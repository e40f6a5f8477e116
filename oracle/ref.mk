# oracle/ref.mk -- build recipe for the UNMODIFIED reference cq, compiled from its
# own sources where they lie under $(REF) (never copied into this repo).
#
# Outputs (all under oracle/_ref/, git-ignored, travel to the GPU box prebuilt):
#   libcqref.so    every reference source except main.c  (Makefile:21-23 "libcq")
#   libcqfront.so  the front end the north_star keeps: tokenizer, parser, utils,
#                  csv_reader (printers/csv_free), date_utils, mmap  -- no evaluator
#   cq_ref         the reference CLI (main.c + libcq objects), the CPU baseline
#   ref_probe      our dump driver (oracle/ref_probe.c) linked against libcqref.so
#   cq_amd_cli     the reference main.c linked with the front end + OUR libcqgpu.so:
#                  the drop-in demonstration (built only when libcqgpu.so exists);
#                  main.o's call of write_csv_file (`-o`, main.c:133) is bound to
#                  libcqgpu's GPU writer cqgpu_write_csv by renaming the undefined
#                  symbol in a copy of the object (objcopy --redefine-sym)
#
# The reference Makefile uses `cc -O2` (Makefile:3); we add -fPIC for the .so.
# Usage: make -f oracle/ref.mk REF=/root/reference
REF      ?= /root/reference
OUT      := oracle/_ref
CC       := gcc
CFLAGS   := -O2 -fPIC -w -I$(REF)/include
EVAL_SRC := $(REF)/src/evaluator.c $(wildcard $(REF)/src/evaluator/*.c)
FRONT_SRC:= $(REF)/src/tokenizer.c $(REF)/src/parser.c $(wildcard $(REF)/src/parser/*.c) \
            $(REF)/src/utils.c $(REF)/src/csv_reader.c $(REF)/src/date_utils.c $(REF)/src/mmap.c
MAIN_SRC := $(REF)/src/main.c

FRONT_OBJ := $(patsubst $(REF)/src/%.c,$(OUT)/obj/%.o,$(FRONT_SRC))
EVAL_OBJ  := $(patsubst $(REF)/src/%.c,$(OUT)/obj/%.o,$(EVAL_SRC))
MAIN_OBJ  := $(OUT)/obj/main.o
GPU_LIB   := cq_amd/lib/libcqgpu.so

TARGETS := $(OUT)/libcqref.so $(OUT)/libcqfront.so $(OUT)/cq_ref $(OUT)/ref_probe
ifneq ($(wildcard $(GPU_LIB)),)
TARGETS += $(OUT)/cq_amd_cli
endif

all: $(TARGETS)

$(OUT)/obj/%.o: $(REF)/src/%.c
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OUT)/libcqref.so: $(FRONT_OBJ) $(EVAL_OBJ)
	$(CC) -shared -o $@ $^ -lm

$(OUT)/libcqfront.so: $(FRONT_OBJ)
	$(CC) -shared -o $@ $^ -lm

$(OUT)/cq_ref: $(MAIN_OBJ) $(FRONT_OBJ) $(EVAL_OBJ)
	$(CC) -o $@ $^ -lm

$(OUT)/ref_probe: oracle/ref_probe.c $(OUT)/libcqref.so
	$(CC) -O2 -I$(REF)/include -o $@ oracle/ref_probe.c -L$(OUT) -lcqref -lm -Wl,-rpath,'$$ORIGIN'

# drop-in: unchanged reference CLI + front end, evaluator (and the -o writer)
# replaced by libcqgpu.so
$(OUT)/obj/main_gpu.o: $(MAIN_OBJ)
	objcopy --redefine-sym write_csv_file=cqgpu_write_csv $< $@

$(OUT)/cq_amd_cli: $(OUT)/obj/main_gpu.o $(FRONT_OBJ) $(GPU_LIB)
	$(CC) -o $@ $(OUT)/obj/main_gpu.o $(FRONT_OBJ) -Lcq_amd/lib -lcqgpu -lm \
	    -Wl,-rpath,'$$ORIGIN/../../cq_amd/lib'

clean:
	rm -rf $(OUT)

.PHONY: all clean
