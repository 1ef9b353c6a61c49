/* TEST INFRASTRUCTURE: include/rclone_crypt_gpu.h must compile as strict C11 (cgo compiles the
 * preamble of a binding as C), with every type a binding touches complete and laid out as the
 * library expects. */
#include "../../include/rclone_crypt_gpu.h"

_Static_assert(sizeof(xs_block_desc) == 48, "xs_block_desc");
_Static_assert(sizeof(xs_md5_desc) == 64, "xs_md5_desc");
_Static_assert(sizeof(xs_name_desc) == 16, "xs_name_desc");
_Static_assert(sizeof(rc_reader) == 4 * sizeof(void *), "rc_reader");
_Static_assert(XS_BLOCK_SIZE == XS_BLOCK_DATA + XS_BLOCK_HDR, "block sizes");

int header_check_dummy(void);
int header_check_dummy(void) { return RC_USER_BASE + XS_OK; }
