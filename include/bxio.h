/*
 * bxio.h — host-side MOT I/O of libbxassoc.so: the detection / embedding text files BoxMOT's
 * evaluation writes and reads, and its MOT-challenge result rows.
 *
 * Reference interfaces replaced (file:line in muntherr/boxmot @ /root/reference):
 *   bx_txt_shape / bx_txt_read   np.loadtxt(path, comments="#") of the det / emb files
 *                                boxmot/utils/dataloaders/MOT17.py:147-153 (written by
 *                                boxmot/engine/val.py:157-187 with np.savetxt(fmt='%f'))
 *   bx_mot_format                convert_to_mot_format (numpy branch)
 *                                boxmot/engine/utils.py:101-133
 *   bx_mot_write                 write_mot_results, fmt "%d,%d,%d,%d,%d,%d,%d,%d,%.6f"
 *                                boxmot/engine/utils.py:152-173
 * Numbers parse with strtod (correctly rounded, like numpy's float parser) and print with
 * printf's correctly rounded %f, so files and arrays are bit-identical to numpy's.
 * Every function returns a status code of bxassoc.h; bx_last_error explains failures.
 */
#ifndef BXIO_H
#define BXIO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Rows and columns of a whitespace-separated numeric text file; '#' starts a comment.  Every
 * data row must have the same number of columns (np.loadtxt raises otherwise: BX_ERR_SHAPE). */
int bx_txt_shape(const char *path, int64_t *rows, int32_t *cols);
/* Parse it into out[rows][cols] (float64, row-major). */
int bx_txt_read(const char *path, double *out, int64_t rows, int32_t cols);
/* convert_to_mot_format of tracker outputs tracks[n][ncol >= 7] (x1,y1,x2,y2,id,conf,cls,...)
 * at frame frame_idx -> out[n][9] = frame, id, round(l), round(t), round(w), round(h), 1, cls,
 * conf (float64 like the reference's column_stack; ids/classes truncated as astype(int32),
 * ltwh rounded half-to-even). */
int bx_mot_format(const double *tracks, int64_t n, int32_t ncol, int32_t frame_idx, double *out);
/* Append (append != 0) or write rows mot[n][9] as "%d,%d,%d,%d,%d,%d,%d,%d,%.6f" lines. */
int bx_mot_write(const char *path, const double *mot, int64_t n, int32_t append);

#ifdef __cplusplus
}
#endif

#endif /* BXIO_H */
