// Exercises every entry point of libsdktls end to end (linked statically so the ASan/UBSan build
// instruments it too): keys, CSRs with SANs, root and intermediate CAs, signing, chain checks,
// certificate summaries, keystore/truststore PKCS#12 round trips, RS256 signatures and JWTs, and
// the error paths. Exit status 0 = all checks passed.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

extern "C" {
const char* sdktls_last_error(void);
void sdktls_free(void* p);
int sdktls_generate_rsa_key(int bits, char** key_pem);
int sdktls_public_key_pem(const char* key_pem, char** pub_pem);
int sdktls_make_csr(const char* key_pem, const char* subject, const char* sans, char** csr_pem);
int sdktls_self_signed_ca(const char* key_pem, const char* subject, int days, char** out_pem);
int sdktls_sign_csr_ex(const char* ca_key_pem, const char* ca_cert_pem, const char* csr_pem, int days, long serial,
                       int as_ca, char** out_pem);
int sdktls_sign_csr(const char* ca_key_pem, const char* ca_cert_pem, const char* csr_pem, int days, long serial,
                    char** out_pem);
int sdktls_verify_chain(const char* cert_pem, const char* trusted_pem, const char* untrusted_pem);
int sdktls_cert_info(const char* pem, char** json);
int sdktls_pkcs12(const char* key_pem, const char* chain_pem, const char* alias, const char* password,
                  unsigned char** der, int* der_len);
int sdktls_pkcs12_inspect(const unsigned char* der, int der_len, const char* password, int* has_key);
int sdktls_rs256_sign(const char* key_pem, const unsigned char* msg, int len, unsigned char** sig, int* sig_len);
int sdktls_rs256_verify(const char* pub_pem, const unsigned char* msg, int len, const unsigned char* sig,
                        int sig_len);
int sdktls_jwt_rs256(const char* key_pem, const char* claims_json, char** jwt);
}

namespace {

int g_failures = 0;

void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s (last error: %s)\n", what, sdktls_last_error());
    ++g_failures;
  }
}

// Owns one malloc'ed output of the library.
struct Out {
  char* p = nullptr;
  ~Out() { sdktls_free(p); }
  std::string str() const { return p ? std::string(p) : std::string(); }
};

std::string key(int bits) {
  Out k;
  check(sdktls_generate_rsa_key(bits, &k.p) == 0, "generate key");
  return k.str();
}

std::string csr(const std::string& k, const char* subject, const char* sans) {
  Out c;
  check(sdktls_make_csr(k.c_str(), subject, sans, &c.p) == 0, "make csr");
  return c.str();
}

}  // namespace

int main() {
  const std::string root_key = key(2048), inter_key = key(2048), leaf_key = key(2048), other_key = key(2048);

  Out root, other_root;
  check(sdktls_self_signed_ca(root_key.c_str(), "CN=test-root,O=Mesosphere\\, Inc", 30, &root.p) == 0, "root CA");
  check(sdktls_self_signed_ca(other_key.c_str(), "CN=other-root", 30, &other_root.p) == 0, "other root CA");

  // a leaf signed directly by the root
  const std::string leaf_csr = csr(leaf_key, "CN=node-0-server.svc,O=Mesosphere\\, Inc",
                                   "DNS:node-0-server.svc.autoip.dcos.thisdcos.directory,DNS:vip.svc.l4lb.thisdcos.directory");
  Out leaf;
  check(sdktls_sign_csr(root_key.c_str(), root.p, leaf_csr.c_str(), 10, 0, &leaf.p) == 0, "sign leaf");
  check(sdktls_verify_chain(leaf.p, root.p, nullptr) == 1, "leaf verifies against its root");
  check(sdktls_verify_chain(leaf.p, other_root.p, nullptr) == 0, "leaf does not verify against another root");

  Out info;
  check(sdktls_cert_info(leaf.p, &info.p) == 0, "cert info");
  const std::string js = info.str();
  check(js.find("node-0-server.svc.autoip.dcos.thisdcos.directory") != std::string::npos, "SAN in summary");
  check(js.find("serverAuth") != std::string::npos && js.find("clientAuth") != std::string::npos, "EKUs");
  check(js.find("\"is_ca\": false") != std::string::npos, "leaf is no CA");

  // root -> intermediate -> leaf
  const std::string inter_csr = csr(inter_key, "CN=test-intermediate", "");
  Out inter;
  check(sdktls_sign_csr_ex(root_key.c_str(), root.p, inter_csr.c_str(), 20, 1234, 1, &inter.p) == 0, "sign intermediate");
  Out inter_info;
  check(sdktls_cert_info(inter.p, &inter_info.p) == 0 && inter_info.str().find("\"is_ca\": true") != std::string::npos,
        "intermediate is a CA");
  Out leaf2;
  check(sdktls_sign_csr(inter_key.c_str(), inter.p, csr(leaf_key, "CN=leaf2", "DNS:leaf2").c_str(), 5, 0, &leaf2.p) == 0,
        "sign leaf under intermediate");
  check(sdktls_verify_chain(leaf2.p, root.p, inter.p) == 1, "chain through the intermediate verifies");
  check(sdktls_verify_chain(leaf2.p, root.p, nullptr) == 0, "chain without the intermediate fails");

  // keystore (key + chain) and truststore (root only)
  const std::string chain = std::string(leaf.p) + root.p;
  unsigned char* der = nullptr;
  int der_len = 0, has_key = -1;
  check(sdktls_pkcs12(leaf_key.c_str(), chain.c_str(), "default", "notsecure", &der, &der_len) == 0, "keystore");
  check(sdktls_pkcs12_inspect(der, der_len, "notsecure", &has_key) == 2 && has_key == 1, "keystore contents");
  check(sdktls_pkcs12_inspect(der, der_len, "wrong", &has_key) < 0, "keystore rejects a wrong password");
  sdktls_free(der);
  der = nullptr;
  check(sdktls_pkcs12(nullptr, root.p, "dcos-root", "notsecure", &der, &der_len) == 0, "truststore");
  check(sdktls_pkcs12_inspect(der, der_len, "notsecure", &has_key) >= 1 && has_key == 0, "truststore has no key");
  sdktls_free(der);

  // RS256 signatures and a JWT
  Out pub;
  check(sdktls_public_key_pem(leaf_key.c_str(), &pub.p) == 0, "public key");
  const char msg[] = "signing input";
  unsigned char* sig = nullptr;
  int sig_len = 0;
  check(sdktls_rs256_sign(leaf_key.c_str(), reinterpret_cast<const unsigned char*>(msg), sizeof msg - 1, &sig,
                          &sig_len) == 0 && sig_len == 256, "rs256 sign");
  check(sdktls_rs256_verify(pub.p, reinterpret_cast<const unsigned char*>(msg), sizeof msg - 1, sig, sig_len) == 1,
        "rs256 verify");
  check(sdktls_rs256_verify(leaf.p, reinterpret_cast<const unsigned char*>(msg), sizeof msg - 1, sig, sig_len) == 1,
        "rs256 verify with the certificate's key");
  sig[0] ^= 1;
  check(sdktls_rs256_verify(pub.p, reinterpret_cast<const unsigned char*>(msg), sizeof msg - 1, sig, sig_len) == 0,
        "tampered signature fails");
  sdktls_free(sig);
  Out jwt;
  check(sdktls_jwt_rs256(leaf_key.c_str(), "{\"uid\":\"svc\",\"exp\":1}", &jwt.p) == 0, "jwt");
  const std::string token = jwt.str();
  check(std::count(token.begin(), token.end(), '.') == 2, "jwt has three parts");

  // error paths report and leave nothing allocated
  Out bad;
  check(sdktls_make_csr("not a key", "CN=x", "", &bad.p) == -1 && std::strlen(sdktls_last_error()) > 0,
        "bad key is reported");
  check(sdktls_sign_csr(root_key.c_str(), root.p, "not a csr", 1, 0, &bad.p) == -1, "bad CSR is reported");
  check(sdktls_cert_info("garbage", &bad.p) == -1, "bad certificate is reported");
  const unsigned char junk[] = {0x30, 0x03, 0x02, 0x01, 0x00};
  check(sdktls_pkcs12_inspect(junk, sizeof junk, "x", &has_key) < 0, "junk PKCS#12 is reported");
  check(sdktls_pkcs12(nullptr, "no certificates here", "a", "p", &der, &der_len) == -1, "empty chain is reported");
  check(bad.p == nullptr, "failed calls allocate nothing");

  if (g_failures == 0) std::printf("tls tests passed\n");
  return g_failures == 0 ? 0 : 1;
}
