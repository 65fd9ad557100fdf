/*
 * gsr_ply.h -- C ABI of the PLY point-cloud I/O the reference does with the `plyfile` package
 * (absent from this image):
 *
 *   GaussianModel.save_ply        scene/gaussian_model.py:303-321  (x y z nx ny nz f_dc_* f_rest_*
 *                                 opacity scale_* rot_*, float32, binary little-endian)
 *   GaussianModel.load_ply        scene/gaussian_model.py:329-376  (properties found by name,
 *                                 f_rest_* / scale_* / rot* ordered by their numeric suffix)
 *   storePly / fetchPly           scene/dataset_readers.py:120-143 (x y z nx ny nz float32,
 *                                 red green blue uint8)
 *
 * The format is the published PLY 1.0 one as plyfile writes it: "ply", "format
 * binary_little_endian 1.0", "element vertex N", one "property <type> <name>" line per
 * column, "end_header", then N packed rows.  The reader accepts any PLY 1.0 file: ascii,
 * binary_little_endian and binary_big_endian bodies, every scalar type (char/int8 ...
 * double/float64), other elements before or after "vertex" (list properties included),
 * comment and obj_info lines; it converts the requested vertex properties to float32.
 *
 * Host code only (no GPU): the callers move the arrays to and from the device.  Returns 0 or
 * a GSR_ERR_* code (include/gsr.h; GSR_ERR_ARGUMENT also for malformed files and missing
 * properties); gsr_last_error() has the message.
 */
#ifndef GSR_PLY_H_INCLUDED
#define GSR_PLY_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gsr_ply gsr_ply; /* an open file: parsed header, position of the vertex rows */

int gsr_ply_open(const char* path, gsr_ply** out);
void gsr_ply_close(gsr_ply* ply);
long long gsr_ply_vertex_count(const gsr_ply* ply);
int gsr_ply_property_count(const gsr_ply* ply);
/* name of vertex property i (valid until gsr_ply_close) */
const char* gsr_ply_property_name(const gsr_ply* ply, int i);

/* type of vertex property i: *bytes = 1, 2, 4 or 8 and *kind = 'i' (signed), 'u' (unsigned),
   'f' (float), or 'l' for a list property */
int gsr_ply_property_type(const gsr_ply* ply, int i, int* bytes, char* kind);

/* Read n scalar vertex properties in their own types (host byte order) */
int gsr_ply_read_raw(gsr_ply* ply, int n, const char* const* names, void* const* out,
                     const long long* out_stride);

/* Read n vertex properties by name into float32 arrays: element v of property k goes to
   (char*)out[k] + v * out_stride[k] (bytes). */
int gsr_ply_read_float(gsr_ply* ply, int n, const char* const* names, float* const* out,
                       const long long* out_stride);

/* Write a binary little-endian PLY with one vertex element of N rows and n properties.
   types[k] (Python struct codes): 'b' int8, 'B' uint8, 'h' int16, 'H' uint16, 'i' int32, 'I' uint32,
   'f' float32, 'd' float64; the header names them char, uchar, short, ushort, int, uint, float,
   double, as plyfile does.
   Element v of column k is read from (const char*)columns[k] + v * strides[k] (bytes). */
int gsr_ply_write(const char* path, long long N, int n, const char* const* names, const char* types,
                  const void* const* columns, const long long* strides);

#ifdef __cplusplus
}
#endif

#endif /* GSR_PLY_H_INCLUDED */
