/* FP64 operation counters of the instrumented oracle build (test infrastructure; slots: instrument_ir.py) */
#include <string.h>
unsigned long long __grmo_fpc[32];
void grmo_fpcount_get(unsigned long long out[32]) { memcpy(out, __grmo_fpc, sizeof(__grmo_fpc)); }
void grmo_fpcount_reset(void) { memset(__grmo_fpc, 0, sizeof(__grmo_fpc)); }
