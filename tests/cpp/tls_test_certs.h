// tls_test_certs.h — test certificates made at run time with OpenSSL (no
// files: the reference's tools/certificates are not shipped to the GPU box):
// a CA (EC P-256, self-signed) and a server certificate it signs
// (CN=localhost), all PEM.
#ifndef WSG_TLS_TEST_CERTS_H
#define WSG_TLS_TEST_CERTS_H

#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <stdexcept>
#include <string>

struct TestPki {
    std::string ca_pem, server_cert_pem, server_key_pem;
};

namespace tls_test {

inline EVP_PKEY* ec_key()
{
    EVP_PKEY* k = EVP_EC_gen("P-256");
    if (!k)
        throw std::runtime_error("EVP_EC_gen");
    return k;
}

inline std::string pem_of(X509* x)
{
    BIO* b = BIO_new(BIO_s_mem());
    PEM_write_bio_X509(b, x);
    char* p = nullptr;
    const long n = BIO_get_mem_data(b, &p);
    std::string s(p, size_t(n));
    BIO_free(b);
    return s;
}

inline std::string pem_of(EVP_PKEY* k)
{
    BIO* b = BIO_new(BIO_s_mem());
    PEM_write_bio_PrivateKey(b, k, nullptr, nullptr, 0, nullptr, nullptr);
    char* p = nullptr;
    const long n = BIO_get_mem_data(b, &p);
    std::string s(p, size_t(n));
    BIO_free(b);
    return s;
}

inline X509* make_cert(EVP_PKEY* subject_key, const char* cn, X509* issuer, EVP_PKEY* issuer_key, bool ca, long serial)
{
    X509* x = X509_new();
    X509_set_version(x, 2);
    ASN1_INTEGER_set(X509_get_serialNumber(x), serial);
    X509_gmtime_adj(X509_getm_notBefore(x), -3600);
    X509_gmtime_adj(X509_getm_notAfter(x), 3600L * 24 * 30);
    X509_set_pubkey(x, subject_key);
    X509_NAME* name = X509_get_subject_name(x);
    X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>(cn), -1, -1, 0);
    X509_set_issuer_name(x, issuer ? X509_get_subject_name(issuer) : name);
    X509V3_CTX v3;
    X509V3_set_ctx(&v3, issuer ? issuer : x, x, nullptr, nullptr, 0);
    const char* bc = ca ? "critical,CA:TRUE" : "CA:FALSE";
    if (X509_EXTENSION* e = X509V3_EXT_conf_nid(nullptr, &v3, NID_basic_constraints, bc)) {
        X509_add_ext(x, e, -1);
        X509_EXTENSION_free(e);
    }
    if (!ca) {
        if (X509_EXTENSION* e = X509V3_EXT_conf_nid(nullptr, &v3, NID_subject_alt_name, "DNS:localhost")) {
            X509_add_ext(x, e, -1);
            X509_EXTENSION_free(e);
        }
    }
    if (!X509_sign(x, issuer_key, EVP_sha256()))
        throw std::runtime_error("X509_sign");
    return x;
}

} // namespace tls_test

inline TestPki make_test_pki()
{
    using namespace tls_test;
    EVP_PKEY* ca_key = ec_key();
    X509* ca = make_cert(ca_key, "wsg test CA", nullptr, ca_key, true, 1);
    EVP_PKEY* srv_key = ec_key();
    X509* srv = make_cert(srv_key, "localhost", ca, ca_key, false, 2);
    TestPki p{pem_of(ca), pem_of(srv), pem_of(srv_key)};
    X509_free(srv);
    X509_free(ca);
    EVP_PKEY_free(srv_key);
    EVP_PKEY_free(ca_key);
    return p;
}

#endif
