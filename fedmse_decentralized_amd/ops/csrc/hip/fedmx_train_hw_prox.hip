// The FedProx instantiation (batch <= 12) of the helper-wave training kernel
// (fedmx_train_hw.hip) as a code object of its own, so that ops/build.py can
// compile it with the machine scheduler's memory-operation clustering off
// (SOURCE_FLAGS: -mllvm -misched-cluster=false).  Measured on the round-6
// sources, with bit-identical results (scheduling only): FedProx launch 966
// -> 939 us, while the plain and batch > 12 instantiations lose 1-2.5 % with
// the same flag, so they keep the library's flags
// (profiles/r6_fedprox_nocluster.md).  fedmx_train_hw() launches it through
// fedmx_train_hw_prox_launch().
#define FEDMX_HW_PROX_TU 1
#include "fedmx_train_hw.hip"
