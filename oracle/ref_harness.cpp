/*
 * ref_harness.cpp -- extern "C" entry points around the reference's own RX
 * arithmetic (appended after the functions oracle/build_ref.sh extracts from
 * /root/reference/cpuLS.hpp: matrix_readX, shiftOneRow, matrixMultThenSum,
 * findDistSqrd, divideOneRow).
 *
 * TEST INFRASTRUCTURE ONLY.  The glue below re-states the handful of inline
 * lines of firstVector / doOneSymbol that are not separate functions in the
 * reference (DC drop memcpy, conjugate loop, normalise loop); the FFT stage is
 * not here (FFTW3 is absent from the image): callers pass FFT'd symbols.
 */
extern "C" {

/* matrix_readX (cpuLS.hpp:80-117) on a given file. */
void ref_matrix_readX(complexF *X, int K, const char *path) {
    g_ref_pilot_path = path;
    matrix_readX(X, K);
}

/* rotCube (cpuLS.hpp:400-413): the layout change createZeroForcingMatrix
 * applies to its channel cube before the per-subcarrier cgemm calls. */
void ref_rot_cube(complexF *X, int rows, int cols, int users) { rotCube(X, rows, cols, users); }

/* shiftOneRow (cpuLS.hpp:135-149). */
void ref_shift_one_row(complexF *Y, int K) { shiftOneRow(Y, K, 0); }

/* firstVector after its FFT loop (cpuLS.hpp:290-311). */
void ref_ls_post_fft(const complexF *Yfft, complexF *X, int rows, int cols,
                     complexF *Hconj, float *Hsqrd_out) {
    for (int row = 0; row < rows; row++) {
        memcpy(&Hconj[row * (cols - 1)], &Yfft[row * cols + 1], (cols - 1) * sizeof(*Yfft));
        divideOneRow(Hconj, X, cols - 1, row);
    }
    for (int i = 0; i < rows; i++)
        for (int j = 0; j < cols - 1; j++)
            Hconj[i * (cols - 1) + j].imag = -1 * Hconj[i * (cols - 1) + j].imag;
    complexF *Xs = (complexF *)malloc((cols - 1) * sizeof(*Xs));
    findDistSqrd(Hconj, Xs, rows, cols - 1);
    for (int j = 0; j < cols - 1; j++) Hsqrd_out[j] = Xs[j].real;
    free(Xs);
}

/* doOneSymbol after its FFT loop (cpuLS.hpp:354-368). */
void ref_mrc_post_fft(const complexF *Yfft, complexF *Hconj, const float *Hsqrd,
                      int rows, int cols, complexF *Yf) {
    complexF *Ytemp = (complexF *)malloc(rows * (cols - 1) * sizeof(*Ytemp));
    for (int row = 0; row < rows; row++)
        memcpy(&Ytemp[row * (cols - 1)], &Yfft[row * cols + 1], (cols - 1) * sizeof(*Yfft));
    matrixMultThenSum(Ytemp, Hconj, Yf, rows, cols);
    for (int j = 0; j < cols - 1; j++) {
        Yf[j].real = Yf[j].real / Hsqrd[j];
        Yf[j].imag = Yf[j].imag / Hsqrd[j];
    }
    shiftOneRow(Yf, cols - 1, 0);
    free(Ytemp);
}

}
