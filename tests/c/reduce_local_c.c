/*
 * Pure-C caller of libmpix_redop.so, written the way MPICH's own test
 * test/mpi/coll/reduce_local.c:55-67 exercises MPI_Reduce_local (with its
 * nested check fixed), plus the MPIR_op_function table (mpir_op.h:206) and a
 * MAXLOC on MPI_2INT -- i.e. what a C integrator of the drop-in sees.
 * Device buffers come from hipMalloc; host buffers are used as-is (staged or
 * zero-copy by the library).  Exit status = number of errors.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpix_redop.h"

#define NMAX 32768     /* largest count of the reference test's doubling sweep */

static int check_2i(const int *io, int count, const char *what)
{
    int errs = 0;
    for (int i = 0; i < count; ++i)
        if (io[i] != 2 * i) {
            if (errs < 5)
                fprintf(stderr, "%s: inout[%d] = %d, expected %d\n", what, i, io[i], 2 * i);
            ++errs;
        }
    return errs;
}

int main(void)
{
    int errs = 0;
    int *in = malloc(sizeof(int) * NMAX);
    int *io = malloc(sizeof(int) * NMAX);
    int *d_in, *d_io;
    if (hipMalloc((void **) &d_in, sizeof(int) * NMAX) != hipSuccess ||
        hipMalloc((void **) &d_io, sizeof(int) * NMAX) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    if (MPIX_Redop_init() != MPIX_REDOP_SUCCESS)
        return 1;
    for (int count = 0; count <= NMAX; count = count ? 2 * count : 1) {
        for (int k = 0; k < count; ++k) {
            in[k] = k;
            io[k] = k;
        }
        /* host buffers */
        if (MPIX_Reduce_local(in, io, count, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_SUCCESS)
            ++errs;
        for (int i = 0; i < count; ++i)
            if (in[i] != i)
                ++errs;
        errs += check_2i(io, count, "host");
        /* device buffers */
        for (int i = 0; i < count; ++i)
            io[i] = i;
        hipMemcpy(d_in, in, sizeof(int) * count, hipMemcpyHostToDevice);
        hipMemcpy(d_io, io, sizeof(int) * count, hipMemcpyHostToDevice);
        if (MPIX_Reduce_local(d_in, d_io, count, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_SUCCESS)
            ++errs;
        hipMemcpy(io, d_io, sizeof(int) * count, hipMemcpyDeviceToHost);
        errs += check_2i(io, count, "device");
    }
    /* the op table, called like MPIR_OP_HDL_TO_FN(op)(in, inout, &len, &type) */
    {
        MPIX_Aint len = 1000;
        MPIX_Datatype ty = MPIX_Datatype_internal(MPIX_MPI_INT);
        for (int i = 0; i < len; ++i) {
            in[i] = (i * 7919) % 1000 - 500;
            io[i] = (i * 104729) % 1000 - 500;
        }
        hipMemcpy(d_in, in, sizeof(int) * len, hipMemcpyHostToDevice);
        hipMemcpy(d_io, io, sizeof(int) * len, hipMemcpyHostToDevice);
        MPIX_Op_table[MPIX_MAX & 0xf](d_in, d_io, &len, &ty);
        if (MPIX_Redop_last_error())
            ++errs;
        int *got = malloc(sizeof(int) * len);
        hipMemcpy(got, d_io, sizeof(int) * len, hipMemcpyDeviceToHost);
        for (int i = 0; i < len; ++i)
            if (got[i] != (io[i] > in[i] ? io[i] : in[i]))
                ++errs;
        free(got);
    }
    /* MAXLOC on MPI_2INT: ties keep the minimum loc (opmaxloc.c:20-23) */
    {
        int a[6] = {1, 5, 0, 7, 3, 2}, b[6] = {1, 3, 4, 9, 3, 8};
        int exp[6] = {1, 3, 4, 9, 3, 2};
        if (MPIX_Reduce_local(b, a, 3, MPIX_MPI_2INT, MPIX_MAXLOC) != MPIX_REDOP_SUCCESS)
            ++errs;
        if (memcmp(a, exp, sizeof(a)))
            ++errs;
    }
    /* binding-level error classes */
    if (MPIX_Reduce_local(d_in, d_in, 10, MPIX_MPI_INT, MPIX_SUM) != MPIX_REDOP_ERR_BUFFER)
        ++errs;
    if (MPIX_Reduce_local(d_in, d_io, 10, MPIX_MPI_FLOAT, MPIX_BAND) != MPIX_REDOP_ERR_OP)
        ++errs;
    MPIX_Redop_finalize();
    hipFree(d_in);
    hipFree(d_io);
    free(in);
    free(io);
    printf("%s (%d errors)\n", errs ? "FAILED" : "No Errors", errs);
    return errs;
}
