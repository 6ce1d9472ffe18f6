// ISA of the packed aligner's hot shape alone (k_alignt2<8, 2, true, 6>), for quick inspection of
// register pressure, spills and waits without building the whole engine (~20 s instead of ~4 min):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
//         -o /tmp/isa/at2.s tools/isa_alignt2.hip [-DTAXI2_AT2_CHUNK=16 ...]
#include "../taxi2_amd/csrc/alignt2_kernel.hpp"

void* taxi2_isa_alignt2_entry() { return (void*)&taxi2::k_alignt2<8, 2, true, 6>; }
