/*
 * hiphuff_plugin.h -- the decoder with the reference's plugin signature.
 *
 * The reference harness registers decoders as
 *     struct decoder { void (*decoder_function)(struct CompressedData *,
 *                      struct UnCompressedData *, void *); void *paramdata;
 *                      char *name; }                (framework/decodeUtil.h:14-19)
 * and its GPU decoders have exactly this signature: openclApproach
 * (framework/openclapproach.h:11-13) and fastgpuApproach
 * (framework/fastgpu.h:13-15, extern "C" at framework/fastgpu.cu:140).
 *
 * hipHuffApproach is the drop-in replacement: the reference's main() adds
 *     hip = newDecoder(hipHuffApproach, NULL, "hip");      (cf. mainrun.c:480-488)
 * and evaluate() (decodeUtil.c:30-70) times and byte-checks it unchanged.
 *
 * The struct types are the reference's own (huffdata.h:12-37); this header
 * only forward-declares them so it can be included next to huffdata.h.
 *
 * Behaviour: decodes cd->bits bits of cd->data with cd->tree into
 * uncompressed->data (the caller's buffer of uncompressedsize + 3 bytes,
 * huffdata.c:166-173).  uncompressed->uncompressedsize is not modified
 * (as fastgpuApproach).  On any error it prints a message to stderr and
 * exits with status 1, the reference's failure mode (decodeUtil.c:47-52,
 * fastgpu.cu:16-31).  paramdata must be NULL (the reference passes NULL for
 * its GPU decoders, mainrun.c:483-487).  Device state (tables, workspace) is
 * cached between calls like the reference's lazy OpenCL globals
 * (openclapproach.c:231-234) and released at exit.
 */
#ifndef HIPHUFF_PLUGIN_H_
#define HIPHUFF_PLUGIN_H_

#ifdef __cplusplus
extern "C" {
#endif

struct CompressedData;
struct UnCompressedData;

void hipHuffApproach(struct CompressedData *cd, struct UnCompressedData *uncompressed,
                     void *paramdata);

#ifdef __cplusplus
}
#endif
#endif
