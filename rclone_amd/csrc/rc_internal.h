// Internal definition of the rc_cipher handle shared by cipher.cpp (data path) and names.cpp
// (file-name path): the counterpart of backend/crypt/cipher.go's Cipher struct (:172-184).
#pragma once
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rclone_crypt_gpu.h"
#include "xs_aes.h"
#include "xs_topo.h"

namespace xs {
void set_error(const char* fmt, ...);  // thread-local message returned by xs_last_error
// Devices a process spreads its work over: RCLONE_AMD_DEVICES ("0,1,2,3"; repeats allowed),
// else RCLONE_AMD_DEVICE, else the local rank's device when LOCAL_RANK is set (one process per
// GPU), else every visible device.
std::vector<int> default_devices();

}  // namespace xs

struct rc_cipher {
  uint8_t data_key[32] = {0};   // dataKey
  uint8_t name_key[32] = {0};   // nameKey
  uint8_t name_tweak[16] = {0}; // nameTweak
  xs::aes::EmeKey eme{};        // block: aes.NewCipher(nameKey) round keys + tweak (EME kernel argument)
  int32_t mode = RC_NAME_STANDARD;     // mode NameEncryptionMode
  int32_t name_enc = RC_ENC_BASE32;    // fileNameEnc
  bool dir_name_encrypt = true;        // dirNameEncrypt
  std::string encrypted_suffix = ".bin";  // encryptedSuffix
  bool pass_bad_blocks = false;
  rc_reader rand{};  // c.cryptoRand; read == NULL -> OS random
  uint32_t batch_blocks = 64;  // read-ahead cap per GPU submission (rc_cipher_set_batch_blocks)
  uint32_t first_blocks = 1;   // first refill of a stream / after a seek (rc_cipher_set_readahead)
  uint32_t growth = 0;         // refill growth factor; 0 = adaptive (rc_cipher_set_readahead_growth)
  xs_pool* pool = nullptr;     // engines; nullptr -> the process-wide pool
  std::mutex rand_mu;
};

// The name cipher's GPU side (names_gpu.cpp), called by the host half (names.cpp).
namespace rcn {
struct EmeDev;
// Lock a name engine whose pinned staging holds >= bytes; *host = that staging (nullptr on error).
EmeDev* eme_acquire(size_t bytes, uint8_t** host);
// host[0:total] -> device, EME in place over the names (descriptors at desc_off), data back.
int32_t eme_run(EmeDev* dev, bool encrypt, const rc_cipher* c, size_t desc_off, size_t ndesc, size_t data_bytes,
                size_t total, double* ms);
void eme_release(EmeDev* dev);
}  // namespace rcn
