/*
 * dfwfm_ingest.h -- C ABI of the native data ingest (libdfwfm_ingest.so, host only).
 *
 * Replaces the reference's pure-Python readers of the step before the forward
 * (SURVEY.md §8f row 4): utils/data_preprocess.py `read_data` (:54-72: one
 * "label,v_1,...,v_C" CSV line per sample; the columns in num_list are numerical values,
 * every other column but the label is a categorical index) and `load_category_index`
 * (:18-26: "field,value,index" lines -> one dict per field, feature_sizes = distinct
 * values + 1).  The file is memory-mapped and parsed by n_threads threads straight into
 * caller-owned arrays (e.g. numpy, or pinned host buffers for the device copy).
 *
 * Token rules follow Python's: a row is the line with surrounding whitespace stripped,
 * split on ','; labels and indices parse like int() (optional sign and surrounding
 * blanks, decimal digits), values like float() (decimal / exponent / inf / nan).
 * Empty lines are skipped; any other malformed token or a row whose column count differs
 * from the first row's is an error naming the 1-based line (the reference raises
 * ValueError / builds a ragged array).  Status codes as dfwfm.h (0 ok, negative error),
 * message from dfwfm_ingest_last_error().
 */
#ifndef DFWFM_INGEST_H
#define DFWFM_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dfwfm_csv dfwfm_csv;

/* Maps the file and counts its non-empty rows and the columns of the first one. */
int dfwfm_csv_open(const char* path, int32_t n_threads, dfwfm_csv** out, int64_t* n_rows, int32_t* n_cols);

/* Parses every row.  is_numerical[c] (c in [0, n_cols)) marks value columns; column 0 is the label.
 * labels [n_rows] int64; values [n_rows][#numerical] float64 (Python float); indices
 * [n_rows][n_cols - 1 - #numerical] int64, columns in file order. */
int dfwfm_csv_parse(dfwfm_csv* h, const uint8_t* is_numerical, int64_t* labels, double* values, int64_t* indices,
                    int32_t n_threads);

void dfwfm_csv_close(dfwfm_csv* h);

/* Feature map: counts[f] = number of distinct values of field f (lines "field,value,index" with
 * field - feature_dim_start in [0, dim); later duplicates overwrite, as dict assignment). */
int dfwfm_feature_map_counts(const char* path, int32_t feature_dim_start, int32_t dim, int64_t* counts);

const char* dfwfm_ingest_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DFWFM_INGEST_H */
