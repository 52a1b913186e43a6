// rx_species.h — the species counts the device path instantiates, and their translation units.
//
// The reference reads any mixture (Common/src/Framework/reacting_model_library.cpp:1520-1586); the device kernels
// are templates on the species count NS (register arrays, unrolled Stefan-Maxwell / chemistry loops), instantiated for
// every NS of RX_FOR_SPECIES. To keep the build parallel, rx_kernels.hip and rx_bc.hip are compiled once per species
// count with -DRX_NS=<ns> (the Makefile's NS_LIST, which must match RX_FOR_SPECIES) and once with RX_NS = 0:
//   RX_NS = ns: only the species launchers, named RX_NSFN(f) = f_ns<ns>, whose RX_DNS_SWITCH instantiates NS = ns
//               for both dimensions;
//   RX_NS = 0:  everything that does not depend on NS, and the dispatchers (RX_NS_DISPATCH) that call f_ns<ns> by
//               the context's species count.
#pragma once

#ifndef RX_NS
#define RX_NS 0
#endif

// NS = 3 .. 9: the reference's 3-species air and every subset of its 9-species jet mixture that keeps the jet's fuel
// and oxidizer (C4H6, H2O, O2, ...: Test_Cases/TURBOLENT/*/Mixture); nVar = NS + nDim + 2 is then 7 .. 14, the block
// sizes RX_NV_SWITCH instantiates
#define RX_FOR_SPECIES(X, a, b) X(a, b, 3) X(a, b, 4) X(a, b, 5) X(a, b, 6) X(a, b, 7) X(a, b, 8) X(a, b, 9)
constexpr int kMinSpecies = 3, kMaxSpecies = 9;

#define RX_NS_CAT2(a, b) a##_ns##b
#define RX_NS_CAT(a, b) RX_NS_CAT2(a, b)
#define RX_NSFN(f) RX_NS_CAT(f, RX_NS)

#if RX_NS
// the species translation unit: NS = RX_NS in 2-D and 3-D
#define RX_DNS_SWITCH(nd, ns, CALL)                     \
  if ((ns) != RX_NS) return RX_ERR_ARG;                 \
  if ((nd) == 2) {                                      \
    constexpr int NS_ = RX_NS, ND_ = 2;                 \
    CALL;                                               \
  } else if ((nd) == 3) {                               \
    constexpr int NS_ = RX_NS, ND_ = 3;                 \
    CALL;                                               \
  } else {                                              \
    return RX_ERR_ARG;                                  \
  }
#endif

// int name params, calling name_ns<ctx->ns> args
#define RX_NS_PROTO(name, params, ns) int name##_ns##ns params;
#define RX_NS_CASE(name, args, ns) \
  case ns:                         \
    return name##_ns##ns args;
#define RX_NS_DISPATCH(name, params, args)     \
  RX_FOR_SPECIES(RX_NS_PROTO, name, params)    \
  int name params {                            \
    switch (ctx->ns) {                         \
      RX_FOR_SPECIES(RX_NS_CASE, name, args)   \
      default:                                 \
        return RX_ERR_ARG;                     \
    }                                          \
  }
