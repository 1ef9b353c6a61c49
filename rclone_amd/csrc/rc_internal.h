// Internal definition of the rc_cipher handle shared by cipher.cpp (data path) and names.cpp
// (file-name path): the counterpart of backend/crypt/cipher.go's Cipher struct (:172-184).
#pragma once
#include <mutex>
#include <string>

#include "../../include/rclone_crypt_gpu.h"
#include "xs_aes.h"

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
  uint32_t batch_blocks = 64;
  std::mutex rand_mu;
};
