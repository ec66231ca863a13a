# Host-side sanitizer builds of the C-ABI libraries: the host
# C++ (redop_capi.cpp, coll_capi.cpp) instrumented, the gfx950 kernel objects
# of the regular build linked as they are, and the pure-C driver
# tests/c/coll_host_sanitize.c on top.  CPU only: the driver runs the
# schedules on the host-memory transport with the oracle's combine.
#   make -f sanitize.mk SAN=asan   # AddressSanitizer + UndefinedBehaviorSanitizer
#   make -f sanitize.mk SAN=tsan   # ThreadSanitizer (the in-process transport's mailbox)
# Outputs in build/$(SAN)/ (git-ignored); run build/$(SAN)/coll_host_sanitize.
SAN ?= asan
CXX ?= g++
CC ?= gcc
ifeq ($(SAN),tsan)
SANFLAGS = -fsanitize=thread
else
SANFLAGS = -fsanitize=address,undefined -fno-sanitize-recover=undefined
endif
OUT = build/$(SAN)
ORACLE = ../../oracle/build
HOSTFLAGS = -O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -Wall -D__HIP_PLATFORM_AMD__ \
            -I/opt/rocm/include -I../../include -I.
KOBJS = build/inst_int.o build/inst_fp.o build/inst_pair.o

all: $(OUT)/coll_host_sanitize

$(KOBJS):
	$(MAKE) -s

$(OUT)/%.o: %.cpp ../../include/mpix_redop.h ../../include/mpix_coll.h redop_dispatch.h
	@mkdir -p $(OUT)
	$(CXX) $(HOSTFLAGS) $(SANFLAGS) -c $< -o $@

$(OUT)/libmpix_redop.so: $(OUT)/redop_capi.o $(KOBJS)
	$(CXX) -shared -fPIC $(SANFLAGS) -o $@ $^ -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-soname,libmpix_redop.so -Wl,-rpath,/opt/rocm/lib

$(OUT)/libmpix_coll.so: $(OUT)/coll_capi.o $(OUT)/libmpix_redop.so
	$(CXX) -shared -fPIC $(SANFLAGS) -o $@ $(OUT)/coll_capi.o -L$(OUT) -lmpix_redop \
	    -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-soname,libmpix_coll.so \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib

$(ORACLE)/liboracle_redop.so:
	$(MAKE) -s -C ../../oracle

$(OUT)/coll_host_sanitize: ../../tests/c/coll_host_sanitize.c $(OUT)/libmpix_coll.so \
                           $(ORACLE)/liboracle_redop.so
	$(CC) -std=gnu11 -O1 -g -fno-omit-frame-pointer -Wall $(SANFLAGS) -D__HIP_PLATFORM_AMD__ \
	    -I../../include -I/opt/rocm/include -o $@ $< -L$(OUT) -lmpix_coll -lmpix_redop \
	    -L$(ORACLE) -loracle_redop -lpthread \
	    -Wl,-rpath,$(abspath $(OUT)) -Wl,-rpath,$(abspath $(ORACLE)) -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf $(OUT)

.PHONY: all clean
