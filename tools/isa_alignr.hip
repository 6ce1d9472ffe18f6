// ISA of the row-shared aligner's hot shape alone (k_alignr<8, 2, 5>), for quick inspection of
// register pressure, spills and the step loops without building the whole engine:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
//         -o /tmp/isa/ar.s tools/isa_alignr.hip [-DTAXI2_AR_SKIP=0 ...]
//   python tools/step_isa.py /tmp/isa/ar.s --kernel k_alignrILi8ELi2ELi5E
#include "../taxi2_amd/csrc/alignr_kernel.hpp"

void* taxi2_isa_alignr_entry() { return (void*)&taxi2::k_alignr<8, 2, 5>; }
