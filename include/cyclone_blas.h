/* cyclone_blas.h -- libcyclone_blas.so: netlib-compatible BLAS on MI355X.
 *
 * Layer 1 of the boundary: the per-call symbols that
 * dev.ludovic.netlib's native BLAS binds (JNIBLAS -> the Fortran ABI) when
 * the executor JVM runs with
 *   -Ddev.ludovic.netlib.blas.nativeLibPath=/path/to/libcyclone_blas.so
 * (docs/ml-linalg-guide.md:59-75).  Every routine below replaces one
 * NetlibBLAS method that the reference calls through BLAS.nativeBLAS /
 * BLAS.getBLAS(n) (mllib-local/src/main/scala/org/apache/spark/ml/linalg/
 * BLAS.scala:42-55):
 *
 *   dgemm_   ml/linalg/BLAS.scala:422,  mllib/linalg/BLAS.scala:404
 *   dgemv_   ml/linalg/BLAS.scala:630
 *   dspr_    ml/linalg/BLAS.scala:284,  mllib/linalg/BLAS.scala:268
 *            (RowMatrix Gramian / covariance per-row rank-1 update)
 *   dsyr_    ml/linalg/BLAS.scala:336,  mllib/linalg/BLAS.scala:319
 *   daxpy_   ml/linalg/BLAS.scala:85,116
 *   ddot_    ml/linalg/BLAS.scala:145
 *   dscal_   ml/linalg/BLAS.scala:240,242,390,496,555,791
 *   dspmv_   ml/linalg/BLAS.scala:272 (bound to javaBLAS there; exported for
 *            completeness)
 *   dger_, dcopy_, dnrm2_  (NetlibBLAS surface; no hot caller)
 *
 * Contract (netlib): host pointers, column-major, int32 dimensions, all
 * Fortran arguments by reference, synchronous return.  Operands are staged
 * through a per-thread device scratch on a per-thread HIP stream, so the
 * library is reentrant across executor threads.  Argument errors follow
 * XERBLA's parameter numbering: the call returns without touching its
 * outputs and the message (" ** On entry to DGEMM  parameter number 8 had an
 * illegal value") is available from libcyclone's cyc_last_error().
 *
 * This layer pays a PCIe round trip per call; it exists so that every
 * netlib call site works unchanged.  The hot paths bind cyclone.h's
 * device-resident entry points instead.
 */
#ifndef CYCLONE_BLAS_H
#define CYCLONE_BLAS_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Fortran ABI (netlib reference BLAS 3.x names) */
void dgemm_(const char* transa, const char* transb, const int* m, const int* n, const int* k,
            const double* alpha, const double* a, const int* lda, const double* b,
            const int* ldb, const double* beta, double* c, const int* ldc);
void dgemv_(const char* trans, const int* m, const int* n, const double* alpha, const double* a,
            const int* lda, const double* x, const int* incx, const double* beta, double* y,
            const int* incy);
void dspr_(const char* uplo, const int* n, const double* alpha, const double* x, const int* incx,
           double* ap);
void dsyr_(const char* uplo, const int* n, const double* alpha, const double* x, const int* incx,
           double* a, const int* lda);
void dger_(const int* m, const int* n, const double* alpha, const double* x, const int* incx,
           const double* y, const int* incy, double* a, const int* lda);
void dspmv_(const char* uplo, const int* n, const double* alpha, const double* ap,
            const double* x, const int* incx, const double* beta, double* y, const int* incy);
double ddot_(const int* n, const double* x, const int* incx, const double* y, const int* incy);
void daxpy_(const int* n, const double* alpha, const double* x, const int* incx, double* y,
            const int* incy);
void dscal_(const int* n, const double* alpha, double* x, const int* incx);
void dcopy_(const int* n, const double* x, const int* incx, double* y, const int* incy);
double dnrm2_(const int* n, const double* x, const int* incx);

/* ---- CBLAS (CblasRowMajor = 101, CblasColMajor = 102; CblasNoTrans = 111,
 * CblasTrans = 112, CblasConjTrans = 113; CblasUpper = 121, CblasLower = 122) */
void cblas_dgemm(int layout, int transa, int transb, int m, int n, int k, double alpha,
                 const double* a, int lda, const double* b, int ldb, double beta, double* c,
                 int ldc);
void cblas_dgemv(int layout, int trans, int m, int n, double alpha, const double* a, int lda,
                 const double* x, int incx, double beta, double* y, int incy);
void cblas_dspr(int layout, int uplo, int n, double alpha, const double* x, int incx, double* ap);
void cblas_dsyr(int layout, int uplo, int n, double alpha, const double* x, int incx, double* a,
                int lda);
void cblas_dger(int layout, int m, int n, double alpha, const double* x, int incx,
                const double* y, int incy, double* a, int lda);
double cblas_ddot(int n, const double* x, int incx, const double* y, int incy);
void cblas_daxpy(int n, double alpha, const double* x, int incx, double* y, int incy);
void cblas_dscal(int n, double alpha, double* x, int incx);
void cblas_dcopy(int n, const double* x, int incx, double* y, int incy);
double cblas_dnrm2(int n, const double* x, int incx);

#ifdef __cplusplus
}
#endif

#endif /* CYCLONE_BLAS_H */
