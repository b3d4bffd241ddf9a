// f4_prof.cpp — host-only profile harness of the f4 ingest path (C3's
// publication: 2,080 adj + 208k prefix keys through
// LsdbIngest::processPublication and the per-key updateKeyInLsdb loop), for
// gprof / timing on the CPU (no device: linked with tests/asan/ogs_stub.cpp).
//   make -C tools/f4prof && tools/f4prof/f4_prof [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "decision.h"
#include "lsdb_codec.h"
#include "lsdb_gen.h"

using namespace openr_amd;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  topogen::FabricOpts o;  // workloads.C3_OPTS
  o.pods = 32;
  o.planes = 8;
  o.sswPerPlane = 36;
  o.rswPerPod = 48;
  o.full = true;
  o.prefixesPerNode = 100;
  o.prefixSeed = 0xC3;
  auto g = topogen::fabric(o);
  topogen::applyOverloads(g, 0, 0, 0x0F);
  topogen::PrefixMix m;
  m.seed = 0x3F;
  topogen::applyPrefixMix(g, m);
  std::vector<std::string> keys, vals;
  lsdbPublication(g, keys, vals);
  const size_t nAdj = g.adjDbs.size();
  std::vector<PublicationKeyVal> pub(keys.size());
  for (size_t i = 0; i < keys.size(); ++i) pub[i] = PublicationKeyVal{keys[i], vals[i]};
  std::sort(pub.begin(), pub.end(),
            [](const PublicationKeyVal& a, const PublicationKeyVal& b) { return a.key < b.key; });
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  for (int r = 0; r < reps; ++r) {
    double tp, ta, tq;
    {
      AreaLinkStates als;
      PrefixState ps0;
      LsdbIngest ing0("test_node", {g.area});
      DecisionPendingUpdates pending("test_node");
      auto p0 = std::chrono::steady_clock::now();
      ing0.processPublication(g.area, als, ps0, pub, {}, pending);
      tp = ms(p0, std::chrono::steady_clock::now());
    }
    {
      LinkState ls(g.area, "test_node");
      PrefixState ps;
      LsdbIngest ing("test_node", {g.area});
      auto t0 = std::chrono::steady_clock::now();
      for (size_t i = 0; i < nAdj; ++i) ing.updateKeyInLsdb(g.area, ls, ps, keys[i], std::string_view(vals[i]));
      auto t1 = std::chrono::steady_clock::now();
      for (size_t i = nAdj; i < keys.size(); ++i) {
        ing.updateKeyInLsdb(g.area, ls, ps, keys[i], std::string_view(vals[i]));
      }
      auto t2 = std::chrono::steady_clock::now();
      ta = ms(t0, t1);
      tq = ms(t1, t2);
    }
    // the prefix keys' decode alone, then the apply of the decoded keys
    double td, tapp;
    {
      LinkState ls(g.area, "test_node");
      PrefixState ps;
      LsdbIngest ing("test_node", {g.area});
      std::vector<LsdbIngest::Decoded> dec;
      dec.reserve(keys.size() - nAdj);
      auto t0 = std::chrono::steady_clock::now();
      for (size_t i = nAdj; i < keys.size(); ++i) {
        dec.push_back(LsdbIngest::decodeKey(keys[i], std::string_view(vals[i])));
      }
      auto t1 = std::chrono::steady_clock::now();
      for (size_t i = nAdj; i < keys.size(); ++i) {
        ing.applyDecoded(g.area, ls, ps, keys[i], std::move(dec[i - nAdj]));
      }
      auto t2 = std::chrono::steady_clock::now();
      td = ms(t0, t1);
      tapp = ms(t1, t2);
    }
    std::printf("rep %d: processPublication %.1f ms | per-key: adj %.1f ms + prefix %.1f ms = %.1f"
                " | prefix decode %.1f + apply %.1f\n", r, tp, ta, tq, ta + tq, td, tapp);
  }
  return 0;
}
