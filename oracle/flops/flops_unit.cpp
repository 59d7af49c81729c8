/* Flop-counting build of the CPU oracle (MEASUREMENT INFRASTRUCTURE ONLY): the oracle's C sources
 * compiled as C++ with `double` -> fdbl (fcount.hpp), exporting the same C entry points plus the
 * counter.  Build: make -C oracle flops.  Run single-threaded (OMP_NUM_THREADS=1): the counter is
 * per thread. */
#include "fcount.hpp"

extern "C" {
__thread unsigned long long ur3f_flops = 0;
#include "../ur3e_oracle.c"
#include "../ur3e_oracle_batch.c"
unsigned long long ur3f_get_flops(void) { return ur3f_flops; }
void ur3f_reset_flops(void) { ur3f_flops = 0; }
}
