// Stub kernel of a compiled-program code object (mythril_amd/jit.py).  Its
// device assembly (built once, lib/mg_jit_stub.s) gives every JIT image a
// well-formed kernel descriptor and metadata; the programs and their entry
// table (mg_jit_table) are appended to it as assembly.  Nothing launches it.
#include <hip/hip_runtime.h>

extern "C" __global__ void mg_jit_stub(unsigned int* p) {
    if (p) p[threadIdx.x] = 0;
}
