// libsdktls: the crypto half of TLS provisioning, as a small C ABI over OpenSSL libcrypto.
//
// Reference behaviour (sdk/.../offer/evaluate/security/TLSArtifactsGenerator.java:60-189,
// PEMUtils.java, dcos/clients/ServiceAccountIAMTokenClient.java) implemented in BouncyCastle/JCA
// there; here natively:
//   * RSA-2048 key pairs (PKCS#8 PEM);
//   * PKCS#10 CSRs signed SHA256withRSA carrying the extensionRequest the reference adds:
//     keyUsage=digitalSignature (critical), extendedKeyUsage=clientAuth,serverAuth (critical),
//     subjectAltName=<DNS names> (critical);
//   * a CA: self-signed root and CSR signing that copies the requested extensions (used by the
//     DC/OS CA stand-in and by tests);
//   * PKCS#12 keystores (key + chain, alias "default") and truststores (root CA, alias
//     "dcos-root", tagged with the JDK trusted-certificate attribute so Java's KeyStore sees a
//     trusted entry), password-protected;
//   * RS256 signatures for service-account login JWTs, and verification.
// Every function returns 0 on success / -1 on failure (message via sdktls_last_error()); output
// buffers are malloc'ed and released with sdktls_free().
#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/pkcs12.h>
#include <openssl/rsa.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

thread_local std::string g_error;

int fail(const std::string& what) {
  unsigned long e = ERR_get_error();
  g_error = what;
  if (e != 0) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof buf);
    g_error += ": ";
    g_error += buf;
  }
  ERR_clear_error();
  return -1;
}

template <typename T, void (*F)(T*)>
struct Deleter {
  void operator()(T* p) const { F(p); }
};
using BioPtr = std::unique_ptr<BIO, Deleter<BIO, BIO_free_all>>;
using KeyPtr = std::unique_ptr<EVP_PKEY, Deleter<EVP_PKEY, EVP_PKEY_free>>;
using X509Ptr = std::unique_ptr<X509, Deleter<X509, X509_free>>;
using ReqPtr = std::unique_ptr<X509_REQ, Deleter<X509_REQ, X509_REQ_free>>;
using NamePtr = std::unique_ptr<X509_NAME, Deleter<X509_NAME, X509_NAME_free>>;
using MdCtxPtr = std::unique_ptr<EVP_MD_CTX, Deleter<EVP_MD_CTX, EVP_MD_CTX_free>>;

void free_x509_stack(STACK_OF(X509) * s) { sk_X509_pop_free(s, X509_free); }
void free_ext_stack(STACK_OF(X509_EXTENSION) * s) { sk_X509_EXTENSION_pop_free(s, X509_EXTENSION_free); }

char* dup_string(const std::string& s) {
  char* out = static_cast<char*>(std::malloc(s.size() + 1));
  if (out != nullptr) std::memcpy(out, s.c_str(), s.size() + 1);
  return out;
}

std::string bio_string(BIO* b) {
  BUF_MEM* mem = nullptr;
  BIO_get_mem_ptr(b, &mem);
  return mem != nullptr ? std::string(mem->data, mem->length) : std::string();
}

BioPtr mem_bio(const char* s) { return BioPtr(BIO_new_mem_buf(s, -1)); }

KeyPtr read_private_key(const char* pem) {
  BioPtr b = mem_bio(pem);
  return KeyPtr(b ? PEM_read_bio_PrivateKey(b.get(), nullptr, nullptr, nullptr) : nullptr);
}

KeyPtr read_public_key(const char* pem) {
  BioPtr b = mem_bio(pem);
  if (!b) return KeyPtr();
  KeyPtr k(PEM_read_bio_PUBKEY(b.get(), nullptr, nullptr, nullptr));
  if (k) return k;
  // also accept a certificate
  ERR_clear_error();
  BioPtr b2 = mem_bio(pem);
  X509Ptr c(PEM_read_bio_X509(b2.get(), nullptr, nullptr, nullptr));
  return KeyPtr(c ? X509_get_pubkey(c.get()) : nullptr);
}

X509Ptr read_cert(const char* pem) {
  BioPtr b = mem_bio(pem);
  return X509Ptr(b ? PEM_read_bio_X509(b.get(), nullptr, nullptr, nullptr) : nullptr);
}

std::vector<X509Ptr> read_certs(const char* pem) {
  std::vector<X509Ptr> out;
  BioPtr b = mem_bio(pem);
  if (!b) return out;
  while (X509* c = PEM_read_bio_X509(b.get(), nullptr, nullptr, nullptr)) out.emplace_back(c);
  ERR_clear_error();  // reading stops with a "no start line" error at the end
  return out;
}

// "CN=a,O=Mesosphere\, Inc,L=..." ('\,' escapes a comma inside a value)
NamePtr parse_subject(const char* subject) {
  NamePtr name(X509_NAME_new());
  std::string s(subject ? subject : "");
  std::string field, value, *cur = &field;
  auto flush = [&]() -> bool {
    if (field.empty()) return true;
    bool ok = X509_NAME_add_entry_by_txt(name.get(), field.c_str(), MBSTRING_UTF8,
                                         reinterpret_cast<const unsigned char*>(value.c_str()), -1, -1, 0) == 1;
    field.clear();
    value.clear();
    cur = &field;
    return ok;
  };
  for (size_t i = 0; i < s.size(); ++i) {
    char ch = s[i];
    if (ch == '\\' && i + 1 < s.size()) {
      *cur += s[++i];
    } else if (ch == '=' && cur == &field) {
      cur = &value;
    } else if (ch == ',') {
      if (!flush()) return NamePtr();
    } else {
      *cur += ch;
    }
  }
  if (!flush()) return NamePtr();
  return name;
}

bool add_ext(STACK_OF(X509_EXTENSION) * exts, int nid, const char* value) {
  X509_EXTENSION* e = X509V3_EXT_conf_nid(nullptr, nullptr, nid, value);
  if (e == nullptr) return false;
  sk_X509_EXTENSION_push(exts, e);
  return true;
}

std::string cert_pem(X509* c) {
  BioPtr b(BIO_new(BIO_s_mem()));
  PEM_write_bio_X509(b.get(), c);
  return bio_string(b.get());
}

bool set_random_serial(X509* c, long serial) {
  ASN1_INTEGER* sn = X509_get_serialNumber(c);
  if (serial > 0) return ASN1_INTEGER_set(sn, serial) == 1;
  std::unique_ptr<BIGNUM, Deleter<BIGNUM, BN_free>> bn(BN_new());
  if (!bn || BN_rand(bn.get(), 127, BN_RAND_TOP_ANY, BN_RAND_BOTTOM_ANY) != 1) return false;
  return BN_to_ASN1_INTEGER(bn.get(), sn) != nullptr;
}

std::string b64url(const unsigned char* data, size_t len) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  std::string out;
  size_t i = 0;
  for (; i + 2 < len; i += 3) {
    unsigned v = (data[i] << 16) | (data[i + 1] << 8) | data[i + 2];
    out += tbl[(v >> 18) & 63];
    out += tbl[(v >> 12) & 63];
    out += tbl[(v >> 6) & 63];
    out += tbl[v & 63];
  }
  if (i + 1 == len) {
    unsigned v = data[i] << 16;
    out += tbl[(v >> 18) & 63];
    out += tbl[(v >> 12) & 63];
  } else if (i + 2 == len) {
    unsigned v = (data[i] << 16) | (data[i + 1] << 8);
    out += tbl[(v >> 18) & 63];
    out += tbl[(v >> 12) & 63];
    out += tbl[(v >> 6) & 63];
  }
  return out;
}

}  // namespace

extern "C" {

const char* sdktls_last_error(void) { return g_error.c_str(); }

void sdktls_free(void* p) { std::free(p); }

int sdktls_generate_rsa_key(int bits, char** key_pem) {
  KeyPtr key(EVP_RSA_gen(static_cast<unsigned>(bits > 0 ? bits : 2048)));
  if (!key) return fail("RSA key generation failed");
  BioPtr b(BIO_new(BIO_s_mem()));
  if (PEM_write_bio_PKCS8PrivateKey(b.get(), key.get(), nullptr, nullptr, 0, nullptr, nullptr) != 1)
    return fail("PKCS8 encoding failed");
  *key_pem = dup_string(bio_string(b.get()));
  return 0;
}

int sdktls_public_key_pem(const char* key_pem, char** pub_pem) {
  KeyPtr key = read_private_key(key_pem);
  if (!key) return fail("bad private key");
  BioPtr b(BIO_new(BIO_s_mem()));
  if (PEM_write_bio_PUBKEY(b.get(), key.get()) != 1) return fail("public key encoding failed");
  *pub_pem = dup_string(bio_string(b.get()));
  return 0;
}

int sdktls_make_csr(const char* key_pem, const char* subject, const char* sans, char** csr_pem) {
  KeyPtr key = read_private_key(key_pem);
  if (!key) return fail("bad private key");
  ReqPtr req(X509_REQ_new());
  NamePtr name = parse_subject(subject);
  if (!req || !name) return fail("bad subject");
  X509_REQ_set_version(req.get(), 0);
  X509_REQ_set_subject_name(req.get(), name.get());
  X509_REQ_set_pubkey(req.get(), key.get());
  std::unique_ptr<STACK_OF(X509_EXTENSION), void (*)(STACK_OF(X509_EXTENSION)*)> exts(
      sk_X509_EXTENSION_new_null(), free_ext_stack);
  if (!add_ext(exts.get(), NID_key_usage, "critical,digitalSignature") ||
      !add_ext(exts.get(), NID_ext_key_usage, "critical,clientAuth,serverAuth"))
    return fail("extension encoding failed");
  if (sans != nullptr && sans[0] != '\0') {
    std::string v = std::string("critical,") + sans;
    if (!add_ext(exts.get(), NID_subject_alt_name, v.c_str())) return fail("bad subjectAltName");
  }
  if (X509_REQ_add_extensions(req.get(), exts.get()) != 1) return fail("adding extensionRequest failed");
  if (X509_REQ_sign(req.get(), key.get(), EVP_sha256()) <= 0) return fail("CSR signing failed");
  BioPtr b(BIO_new(BIO_s_mem()));
  PEM_write_bio_X509_REQ(b.get(), req.get());
  *csr_pem = dup_string(bio_string(b.get()));
  return 0;
}

int sdktls_self_signed_ca(const char* key_pem, const char* subject, int days, char** out_pem) {
  KeyPtr key = read_private_key(key_pem);
  if (!key) return fail("bad private key");
  X509Ptr c(X509_new());
  NamePtr name = parse_subject(subject);
  if (!c || !name) return fail("bad subject");
  X509_set_version(c.get(), 2);
  if (!set_random_serial(c.get(), 0)) return fail("serial");
  X509_gmtime_adj(X509_getm_notBefore(c.get()), -3600);
  X509_gmtime_adj(X509_getm_notAfter(c.get()), static_cast<long>(days) * 86400L);
  X509_set_subject_name(c.get(), name.get());
  X509_set_issuer_name(c.get(), name.get());
  X509_set_pubkey(c.get(), key.get());
  X509V3_CTX ctx;
  X509V3_set_ctx(&ctx, c.get(), c.get(), nullptr, nullptr, 0);
  const std::pair<int, const char*> exts[] = {{NID_basic_constraints, "critical,CA:TRUE"},
                                              {NID_key_usage, "critical,keyCertSign,cRLSign,digitalSignature"},
                                              {NID_subject_key_identifier, "hash"}};
  for (const auto& e : exts) {
    X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &ctx, e.first, e.second);
    if (ext == nullptr) return fail("CA extension failed");
    X509_add_ext(c.get(), ext, -1);
    X509_EXTENSION_free(ext);
  }
  if (X509_sign(c.get(), key.get(), EVP_sha256()) <= 0) return fail("CA self-signing failed");
  *out_pem = dup_string(cert_pem(c.get()));
  return 0;
}

// as_ca != 0 issues an intermediate CA (CA extensions replace the requested ones).
int sdktls_sign_csr_ex(const char* ca_key_pem, const char* ca_cert_pem, const char* csr_pem, int days, long serial,
                       int as_ca, char** out_pem) {
  KeyPtr ca_key = read_private_key(ca_key_pem);
  X509Ptr ca = read_cert(ca_cert_pem);
  BioPtr b = mem_bio(csr_pem);
  ReqPtr req(b ? PEM_read_bio_X509_REQ(b.get(), nullptr, nullptr, nullptr) : nullptr);
  if (!ca_key || !ca || !req) return fail("bad CA key, CA certificate or CSR");
  KeyPtr req_key(X509_REQ_get_pubkey(req.get()));
  if (!req_key || X509_REQ_verify(req.get(), req_key.get()) != 1) return fail("CSR signature does not verify");
  X509Ptr c(X509_new());
  X509_set_version(c.get(), 2);
  if (!set_random_serial(c.get(), serial)) return fail("serial");
  X509_gmtime_adj(X509_getm_notBefore(c.get()), -300);
  X509_gmtime_adj(X509_getm_notAfter(c.get()), static_cast<long>(days) * 86400L);
  X509_set_subject_name(c.get(), X509_REQ_get_subject_name(req.get()));
  X509_set_issuer_name(c.get(), X509_get_subject_name(ca.get()));
  X509_set_pubkey(c.get(), req_key.get());
  X509V3_CTX ctx;
  X509V3_set_ctx(&ctx, ca.get(), c.get(), nullptr, nullptr, 0);
  if (as_ca) {
    const std::pair<int, const char*> ca_exts[] = {{NID_basic_constraints, "critical,CA:TRUE,pathlen:0"},
                                                   {NID_key_usage, "critical,keyCertSign,cRLSign,digitalSignature"},
                                                   {NID_subject_key_identifier, "hash"}};
    for (const auto& e : ca_exts) {
      X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &ctx, e.first, e.second);
      if (ext == nullptr) return fail("CA extension failed");
      X509_add_ext(c.get(), ext, -1);
      X509_EXTENSION_free(ext);
    }
  } else {
    std::unique_ptr<STACK_OF(X509_EXTENSION), void (*)(STACK_OF(X509_EXTENSION)*)> exts(
        X509_REQ_get_extensions(req.get()), free_ext_stack);
    for (int i = 0; exts && i < sk_X509_EXTENSION_num(exts.get()); ++i)
      X509_add_ext(c.get(), sk_X509_EXTENSION_value(exts.get(), i), -1);
  }
  X509_EXTENSION* aki = X509V3_EXT_conf_nid(nullptr, &ctx, NID_authority_key_identifier, "keyid:always");
  if (aki != nullptr) {
    X509_add_ext(c.get(), aki, -1);
    X509_EXTENSION_free(aki);
  }
  ERR_clear_error();
  if (X509_sign(c.get(), ca_key.get(), EVP_sha256()) <= 0) return fail("certificate signing failed");
  *out_pem = dup_string(cert_pem(c.get()));
  return 0;
}

int sdktls_sign_csr(const char* ca_key_pem, const char* ca_cert_pem, const char* csr_pem, int days, long serial,
                    char** out_pem) {
  return sdktls_sign_csr_ex(ca_key_pem, ca_cert_pem, csr_pem, days, serial, 0, out_pem);
}

int sdktls_verify_chain(const char* cert_pem, const char* trusted_pem, const char* untrusted_pem) {
  X509Ptr cert = read_cert(cert_pem);
  if (!cert) return fail("bad certificate");
  std::unique_ptr<X509_STORE, Deleter<X509_STORE, X509_STORE_free>> store(X509_STORE_new());
  for (auto& c : read_certs(trusted_pem)) X509_STORE_add_cert(store.get(), c.get());
  std::unique_ptr<STACK_OF(X509), void (*)(STACK_OF(X509)*)> chain(sk_X509_new_null(), free_x509_stack);
  if (untrusted_pem != nullptr)
    for (auto& c : read_certs(untrusted_pem)) sk_X509_push(chain.get(), c.release());
  std::unique_ptr<X509_STORE_CTX, Deleter<X509_STORE_CTX, X509_STORE_CTX_free>> ctx(X509_STORE_CTX_new());
  X509_STORE_CTX_init(ctx.get(), store.get(), cert.get(), chain.get());
  int ok = X509_verify_cert(ctx.get());
  if (ok != 1) {
    g_error = X509_verify_cert_error_string(X509_STORE_CTX_get_error(ctx.get()));
    ERR_clear_error();
    return 0;
  }
  return 1;
}

// JSON summary of a certificate: subject, issuer, serial (hex), notAfter (epoch), DNS SANs, EKUs.
int sdktls_cert_info(const char* pem, char** json) {
  X509Ptr c = read_cert(pem);
  if (!c) return fail("bad certificate");
  auto name_str = [](X509_NAME* n) {
    BioPtr b(BIO_new(BIO_s_mem()));
    X509_NAME_print_ex(b.get(), n, 0, XN_FLAG_RFC2253);
    return bio_string(b.get());
  };
  auto esc = [](const std::string& s) {
    std::string o;
    for (char ch : s) {
      if (ch == '"' || ch == '\\') o += '\\';
      o += ch;
    }
    return o;
  };
  std::string out = "{\"subject\": \"" + esc(name_str(X509_get_subject_name(c.get()))) + "\", \"issuer\": \"" +
                    esc(name_str(X509_get_issuer_name(c.get()))) + "\"";
  std::unique_ptr<BIGNUM, Deleter<BIGNUM, BN_free>> bn(ASN1_INTEGER_to_BN(X509_get_serialNumber(c.get()), nullptr));
  char* hex = BN_bn2hex(bn.get());
  out += std::string(", \"serial\": \"") + hex + "\"";
  OPENSSL_free(hex);
  struct tm t;
  ASN1_TIME_to_tm(X509_get0_notAfter(c.get()), &t);
  out += ", \"not_after\": " + std::to_string(static_cast<long long>(timegm(&t)));
  out += ", \"dns\": [";
  GENERAL_NAMES* gens =
      static_cast<GENERAL_NAMES*>(X509_get_ext_d2i(c.get(), NID_subject_alt_name, nullptr, nullptr));
  for (int i = 0; gens && i < sk_GENERAL_NAME_num(gens); ++i) {
    GENERAL_NAME* g = sk_GENERAL_NAME_value(gens, i);
    if (g->type != GEN_DNS) continue;
    const char* s = reinterpret_cast<const char*>(ASN1_STRING_get0_data(g->d.dNSName));
    out += std::string(i ? ", " : "") + "\"" + esc(std::string(s, ASN1_STRING_length(g->d.dNSName))) + "\"";
  }
  GENERAL_NAMES_free(gens);
  out += "], \"eku\": [";
  EXTENDED_KEY_USAGE* eku =
      static_cast<EXTENDED_KEY_USAGE*>(X509_get_ext_d2i(c.get(), NID_ext_key_usage, nullptr, nullptr));
  for (int i = 0; eku && i < sk_ASN1_OBJECT_num(eku); ++i) {
    out += std::string(i ? ", " : "") + "\"" + OBJ_nid2sn(OBJ_obj2nid(sk_ASN1_OBJECT_value(eku, i))) + "\"";
  }
  EXTENDED_KEY_USAGE_free(eku);
  out += std::string("], \"is_ca\": ") + (X509_check_ca(c.get()) ? "true" : "false") + "}";
  *json = dup_string(out);
  return 0;
}

// key_pem may be null (truststore). chain_pem: end-entity first for keystores; certificates to
// trust for truststores.
int sdktls_pkcs12(const char* key_pem, const char* chain_pem, const char* alias, const char* password,
                  unsigned char** der, int* der_len) {
  std::vector<X509Ptr> certs = read_certs(chain_pem);
  if (certs.empty()) return fail("no certificates");
  KeyPtr key;
  if (key_pem != nullptr && key_pem[0] != '\0') {
    key = read_private_key(key_pem);
    if (!key) return fail("bad private key");
  }
  PKCS12* p12 = nullptr;
  if (key) {
    std::unique_ptr<STACK_OF(X509), void (*)(STACK_OF(X509)*)> ca(sk_X509_new_null(), free_x509_stack);
    for (size_t i = 1; i < certs.size(); ++i) sk_X509_push(ca.get(), X509_dup(certs[i].get()));
    p12 = PKCS12_create(password, alias, key.get(), certs[0].get(), ca.get(), NID_aes_256_cbc, NID_aes_256_cbc,
                        PKCS12_DEFAULT_ITER, PKCS12_DEFAULT_ITER, 0);
  } else {
    // Trusted-certificate bags tagged with Oracle's trustedKeyUsage attribute (anyExtendedKeyUsage),
    // which is what makes the JDK load them as trusted certificate entries.
    std::unique_ptr<STACK_OF(PKCS12_SAFEBAG), void (*)(STACK_OF(PKCS12_SAFEBAG)*)> bags(
        sk_PKCS12_SAFEBAG_new_null(), [](STACK_OF(PKCS12_SAFEBAG) * s) { sk_PKCS12_SAFEBAG_pop_free(s, PKCS12_SAFEBAG_free); });
    std::unique_ptr<ASN1_OBJECT, Deleter<ASN1_OBJECT, ASN1_OBJECT_free>> any_eku(OBJ_txt2obj("2.5.29.37.0", 1));
    for (size_t i = 0; i < certs.size(); ++i) {
      PKCS12_SAFEBAG* bag = PKCS12_SAFEBAG_create_cert(certs[i].get());
      if (bag == nullptr) return fail("cert bag");
      std::string name = certs.size() == 1 ? std::string(alias) : std::string(alias) + "-" + std::to_string(i);
      PKCS12_add_friendlyname_utf8(bag, name.c_str(), -1);
      PKCS12_add1_attr_by_txt(bag, "2.16.840.1.113894.746875.1.1", V_ASN1_OBJECT,
                              reinterpret_cast<const unsigned char*>(any_eku.get()), -1);
      sk_PKCS12_SAFEBAG_push(bags.get(), bag);
    }
    std::unique_ptr<STACK_OF(PKCS7), void (*)(STACK_OF(PKCS7)*)> safes(
        sk_PKCS7_new_null(), [](STACK_OF(PKCS7) * s) { sk_PKCS7_pop_free(s, PKCS7_free); });
    PKCS7* p7 = PKCS12_pack_p7encdata(NID_aes_256_cbc, password, -1, nullptr, 0, PKCS12_DEFAULT_ITER, bags.get());
    if (p7 == nullptr) return fail("encrypting truststore");
    sk_PKCS7_push(safes.get(), p7);
    p12 = PKCS12_add_safes(safes.get(), 0);
    if (p12 != nullptr && PKCS12_set_mac(p12, password, -1, nullptr, 0, PKCS12_DEFAULT_ITER, nullptr) != 1) {
      PKCS12_free(p12);
      p12 = nullptr;
    }
  }
  if (p12 == nullptr) return fail("PKCS12 creation failed");
  unsigned char* buf = nullptr;
  int n = i2d_PKCS12(p12, &buf);
  PKCS12_free(p12);
  if (n <= 0) return fail("PKCS12 encoding failed");
  *der = static_cast<unsigned char*>(std::malloc(n));
  std::memcpy(*der, buf, n);
  OPENSSL_free(buf);
  *der_len = n;
  return 0;
}

// Parses a PKCS#12 blob; returns the number of certificates (>= 0) and whether a key is present.
int sdktls_pkcs12_inspect(const unsigned char* der, int der_len, const char* password, int* has_key) {
  const unsigned char* p = der;
  std::unique_ptr<PKCS12, Deleter<PKCS12, PKCS12_free>> p12(d2i_PKCS12(nullptr, &p, der_len));
  if (!p12) return fail("not a PKCS12 structure");
  if (PKCS12_verify_mac(p12.get(), password, -1) != 1) return fail("bad PKCS12 password");
  EVP_PKEY* key = nullptr;
  X509* cert = nullptr;
  STACK_OF(X509)* ca = nullptr;
  if (PKCS12_parse(p12.get(), password, &key, &cert, &ca) != 1) return fail("PKCS12 parse failed");
  int n = (cert != nullptr ? 1 : 0) + (ca != nullptr ? sk_X509_num(ca) : 0);
  *has_key = key != nullptr;
  EVP_PKEY_free(key);
  X509_free(cert);
  sk_X509_pop_free(ca, X509_free);
  return n;
}

int sdktls_rs256_sign(const char* key_pem, const unsigned char* msg, int len, unsigned char** sig, int* sig_len) {
  KeyPtr key = read_private_key(key_pem);
  if (!key) return fail("bad private key");
  MdCtxPtr ctx(EVP_MD_CTX_new());
  size_t n = 0;
  if (EVP_DigestSignInit(ctx.get(), nullptr, EVP_sha256(), nullptr, key.get()) != 1 ||
      EVP_DigestSign(ctx.get(), nullptr, &n, msg, len) != 1)
    return fail("sign init failed");
  *sig = static_cast<unsigned char*>(std::malloc(n));
  if (EVP_DigestSign(ctx.get(), *sig, &n, msg, len) != 1) {
    std::free(*sig);
    return fail("sign failed");
  }
  *sig_len = static_cast<int>(n);
  return 0;
}

int sdktls_rs256_verify(const char* pub_pem, const unsigned char* msg, int len, const unsigned char* sig,
                        int sig_len) {
  KeyPtr key = read_public_key(pub_pem);
  if (!key) return fail("bad public key");
  MdCtxPtr ctx(EVP_MD_CTX_new());
  if (EVP_DigestVerifyInit(ctx.get(), nullptr, EVP_sha256(), nullptr, key.get()) != 1) return fail("verify init");
  int ok = EVP_DigestVerify(ctx.get(), sig, sig_len, msg, len);
  ERR_clear_error();
  return ok == 1 ? 1 : 0;
}

// Builds a compact RS256 JWT from a JSON claims object.
int sdktls_jwt_rs256(const char* key_pem, const char* claims_json, char** jwt) {
  const char* header = "{\"alg\":\"RS256\",\"typ\":\"JWT\"}";
  std::string signing_input =
      b64url(reinterpret_cast<const unsigned char*>(header), std::strlen(header)) + "." +
      b64url(reinterpret_cast<const unsigned char*>(claims_json), std::strlen(claims_json));
  unsigned char* sig = nullptr;
  int n = 0;
  if (sdktls_rs256_sign(key_pem, reinterpret_cast<const unsigned char*>(signing_input.data()),
                        static_cast<int>(signing_input.size()), &sig, &n) != 0)
    return -1;
  std::string token = signing_input + "." + b64url(sig, n);
  std::free(sig);
  *jwt = dup_string(token);
  return 0;
}

}  // extern "C"
