# Builds the reference SU2 reactive fork directly from its sources under /root/reference
# (no configure/autotools) into oracle/_ref/. Test infrastructure only: the objects are
# used by oracle/ref_harness to emit golden vectors; nothing here ships or is measured.
#
# Serial, no MPI, no CGNS, no AD (su2double == double), exactly as the survey's build.
# solver_direct_reactive.cpp is compiled at -O0: CNumerics::Set_Sigmak has no return
# (SU2_CFD/include/numerics_structure.hpp:525-527) and gcc -O2 treats the inlined path in
# Viscous_Residual as unreachable. -O0 keeps the source byte-identical.
REF   ?= /root/reference
OUT   ?= $(dir $(lastword $(MAKEFILE_LIST)))_ref
CXX   ?= g++
CXXFLAGS ?= -O2 -std=c++14 -w -fPIC
INC = -I$(REF)/Common/include -I$(REF)/SU2_CFD/include -I$(REF)/externals/Eigen -I$(REF)/externals
COMMON_SRC := $(wildcard $(REF)/Common/src/*.cpp) $(wildcard $(REF)/Common/src/Framework/*.cpp) $(wildcard $(REF)/Common/src/Tools/*.cpp)
CFD_SRC    := $(filter-out $(REF)/SU2_CFD/src/SU2_CFD.cpp,$(wildcard $(REF)/SU2_CFD/src/*.cpp))
SRC := $(COMMON_SRC) $(CFD_SRC)
OBJ := $(patsubst $(REF)/%.cpp,$(OUT)/obj/%.o,$(SRC))

all: $(OUT)/libsu2ref.a

$(OUT)/obj/SU2_CFD/src/solver_direct_reactive.o: CXXFLAGS := $(subst -O2,-O0,$(CXXFLAGS))

$(OUT)/obj/%.o: $(REF)/%.cpp
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(INC) -c $< -o $@

$(OUT)/libsu2ref.a: $(OBJ)
	rm -f $@ && ar rcs $@ $^

.PHONY: all

# Golden-vector harness (oracle/ref_harness/harness.cpp, our code) linked against the reference objects.
$(OUT)/harness: $(dir $(lastword $(MAKEFILE_LIST)))ref_harness/harness.cpp $(OUT)/libsu2ref.a
	$(CXX) -O0 -std=c++14 -w $(INC) $< $(OUT)/libsu2ref.a -lstdc++fs -o $@

harness: $(OUT)/harness
.PHONY: harness

# The reference's vendored METIS 5 (externals/metis, with the CPPFLAGS of its m4/metis.m4): the partitioner that
# CPhysicalGeometry::SetColorGrid calls (Common/src/geometry_structure.cpp:11446). tools/edge_cut.py and
# tests/test_partition.py compare rx_partition_graph's edge cut with it; nothing in the product links it.
METIS_DIR := $(REF)/externals/metis
METIS_SRC := $(wildcard $(METIS_DIR)/GKlib/*.c) $(wildcard $(METIS_DIR)/libmetis/*.c)
METIS_OBJ := $(patsubst $(METIS_DIR)/%.c,$(OUT)/obj/metis/%.o,$(METIS_SRC))
METIS_FLAGS := -O2 -fPIC -std=gnu99 -w -D_FILE_OFFSET_BITS=64 -DNDEBUG -DNDEBUG2 -DHAVE_EXECINFO_H -DHAVE_GETLINE \
               -I$(METIS_DIR)/include -I$(METIS_DIR)/GKlib -I$(METIS_DIR)/libmetis

$(OUT)/obj/metis/%.o: $(METIS_DIR)/%.c
	@mkdir -p $(dir $@)
	gcc $(METIS_FLAGS) -c $< -o $@

$(OUT)/libmetis.so: $(METIS_OBJ)
	gcc -shared $^ -o $@ -lm

metis: $(OUT)/libmetis.so
.PHONY: metis
