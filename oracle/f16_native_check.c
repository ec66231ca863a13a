/*
 * ORACLE cross-check -- TEST INFRASTRUCTURE ONLY.
 * The reference built with a compiler that has _Float16 (clang, gcc >= 12)
 * puts MPIR_FLOAT16 in the FLOATING_POINT group (configure.ac:2887-2903,
 * mpir_op_util.h:211-217) and reduces it with native _Float16 arithmetic.
 * gcc 11 here lacks _Float16, so redop_oracle.c restates it in software;
 * this file, compiled with clang, computes the same op with the compiler's
 * native _Float16 so a test can compare the two on every fp16 pair.
 */
#include <stdint.h>
#include <string.h>

/* a[i] = OP(a[i], b[i]) for fp16 bit patterns; op index as mpi.h.in */
void f16_native_reduce(const uint16_t *b, uint16_t *a, long n, int opi)
{
    for (long i = 0; i < n; i++) {
        _Float16 x, y, r;
        memcpy(&x, &a[i], 2);
        memcpy(&y, &b[i], 2);
        switch (opi) {
            case 1: r = (x > y) ? x : y; break;
            case 2: r = (x < y) ? x : y; break;
            case 3: r = x + y; break;
            case 4: r = x * y; break;
            default: return;
        }
        memcpy(&a[i], &r, 2);
    }
}
