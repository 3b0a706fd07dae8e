// Sanitizer driver (ASan/UBSan on the CPU restatement). A standalone
// executable built with -fsanitize=address,undefined from
//   - tests/native/hostcheck.cpp (the device math headers csrc/*.h compiled for the host) and
//   - oracle/edc_oracle.c (the C restatement of the reference algorithm),
// so neither is loaded into Python (no sanitizer runtime preloading). It reads one command per
// line on stdin, arguments as hex, and prints one hex result line; tests/test_sanitizers.py
// compares the results with the Python oracle and the golden fixtures. Test infrastructure only.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

extern "C" {
void hc_fe_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out);
void hc_fe_chain(const uint8_t* a, const uint8_t* b, int k, uint8_t* out);
int hc_decompress(const uint8_t* enc, uint8_t* out);
int hc_point_ops(const uint8_t* a, const uint8_t* b, uint8_t* sum, uint8_t* dbl, uint8_t* madd, uint8_t* cof);
void hc_sha512(const uint8_t* head0, const uint8_t* head1, const uint8_t* msg, uint64_t mlen, uint8_t* out);
void hc_challenge(const uint8_t* R, const uint8_t* A, const uint8_t* msg, uint64_t mlen, uint8_t* out);
void hc_sc_reduce_wide(const uint8_t* x64, uint8_t* out);
void hc_sc_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out);
int hc_sc_is_canonical(const uint8_t* s);
void hc_chacha_block(const uint8_t* key, uint64_t counter, uint8_t* out);
int oc_batch_verify(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                    const uint8_t* z_seed, uint8_t* check8, int* evaluated);
int oc_verify(const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, size_t mlen);
}

static std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> v;
  if (s == "-") return v;
  for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back((uint8_t)strtoul(s.substr(i, 2).c_str(), nullptr, 16));
  return v;
}

static void put(const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) printf("%02x", p[i]);
}

// exact-size heap copy, so ASan sees any read past the argument's end
static uint8_t* dup(const std::vector<uint8_t>& v) {
  uint8_t* p = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (!v.empty()) memcpy(p, v.data(), v.size());
  return p;
}

int main() {
  char* line = nullptr;
  size_t cap = 0;
  while (getline(&line, &cap, stdin) > 0) {
    std::vector<std::string> tok;
    for (char* t = strtok(line, " \n"); t; t = strtok(nullptr, " \n")) tok.push_back(t);
    if (tok.empty()) continue;
    const std::string& c = tok[0];
    uint8_t out[256];
    if (c == "fe") {                  // fe op a b
      auto a = unhex(tok[2]), b = unhex(tok[3]);
      hc_fe_op(atoi(tok[1].c_str()), a.data(), b.data(), out);
      put(out, 32);
    } else if (c == "chain") {        // chain a b k
      auto a = unhex(tok[1]), b = unhex(tok[2]);
      hc_fe_chain(a.data(), b.data(), atoi(tok[3].c_str()), out);
      put(out, 32);
    } else if (c == "dec") {          // dec enc
      auto e = unhex(tok[1]);
      int ok = hc_decompress(e.data(), out);
      printf("%d ", ok);
      put(out, 64);
    } else if (c == "pt") {           // pt e1 e2
      auto a = unhex(tok[1]), b = unhex(tok[2]);
      int ok = hc_point_ops(a.data(), b.data(), out, out + 32, out + 64, out + 96);
      printf("%d ", ok);
      put(out, 128);
    } else if (c == "sha" || c == "chal") {   // sha R A|- M|-
      auto R = unhex(tok[1]), A = unhex(tok[2]), M = unhex(tok[3]);
      uint8_t* m = dup(M);
      if (c == "sha") {
        hc_sha512(R.data(), A.empty() ? nullptr : A.data(), m, M.size(), out);
        put(out, 64);
      } else {
        hc_challenge(R.data(), A.data(), m, M.size(), out);
        put(out, 32);
      }
      free(m);
    } else if (c == "scw") {          // scw x64
      auto x = unhex(tok[1]);
      hc_sc_reduce_wide(x.data(), out);
      put(out, 32);
    } else if (c == "sco") {          // sco op a b
      auto a = unhex(tok[2]), b = unhex(tok[3]);
      hc_sc_op(atoi(tok[1].c_str()), a.data(), b.data(), out);
      put(out, 32);
    } else if (c == "canon") {        // canon s
      auto s = unhex(tok[1]);
      printf("%d", hc_sc_is_canonical(s.data()));
    } else if (c == "chacha") {       // chacha key ctr
      auto k = unhex(tok[1]);
      hc_chacha_block(k.data(), strtoull(tok[2].c_str(), nullptr, 10), out);
      put(out, 64);
    } else if (c == "obv") {          // obv zseed vks sigs arena off0,off1,...
      auto z = unhex(tok[1]), vk = unhex(tok[2]), sg = unhex(tok[3]), ar = unhex(tok[4]);
      std::vector<uint64_t> off;
      for (char* t = strtok(&tok[5][0], ","); t; t = strtok(nullptr, ",")) off.push_back(strtoull(t, nullptr, 10));
      const size_t n = off.size() - 1;
      uint8_t *pv = dup(vk), *ps = dup(sg), *pm = dup(ar);
      uint64_t* po = (uint64_t*)malloc(off.size() * sizeof(uint64_t));
      memcpy(po, off.data(), off.size() * sizeof(uint64_t));
      int ev = 0;
      int rc = oc_batch_verify(n, pv, ps, pm, po, z.data(), out, &ev);
      printf("%d %d ", rc, ev);
      put(out, 32);
      free(pv); free(ps); free(pm); free(po);
    } else if (c == "ov") {           // ov vk sig msg|-
      auto vk = unhex(tok[1]), sg = unhex(tok[2]), M = unhex(tok[3]);
      uint8_t* m = dup(M);
      printf("%d", oc_verify(vk.data(), sg.data(), m, M.size()));
      free(m);
    } else {
      printf("?");
    }
    printf("\n");
    fflush(stdout);
  }
  free(line);
  return 0;
}
