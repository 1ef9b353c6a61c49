/* TEST INFRASTRUCTURE: stand-in for the _cgo_export.h that cgo generates for
 * integration/gpucipher/gpucipher.go -- the C prototypes of its //export functions, with the
 * parameter types cgo derives from the Go signatures (C.uintptr_t, *C.uint8_t, C.int64_t, ...).
 * tests/native/c_client.c implements them in C the way the Go functions behave. */
#include <stdint.h>

#include "rclone_crypt_gpu.h"

extern int64_t goRead(uintptr_t h, uint8_t *p, int64_t n, int32_t *errp);
extern int32_t goClose(uintptr_t h);
extern int32_t goRangeSeek(uintptr_t h, int64_t offset, int32_t whence, int64_t limit);
extern int32_t goOpen(uintptr_t h, int64_t offset, int64_t limit, rc_reader *out);
