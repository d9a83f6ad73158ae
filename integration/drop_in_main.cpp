// drop_in_main.cpp -- the reference's own Model (model.cpp, gguf.cpp compiled
// unchanged) driving the MI355X kernels through integration/ops_mi355x.cpp.
// A minimal stand-in for main.cpp's greedy loop (main.cpp:160-224):
//   dropin_mi355x <model.gguf>[,<model2.gguf>...] <n_decode> <tok0> [tok1 ...]
// Several comma-separated files are run one after another in the same
// process, each with its own GGUFFile + Model (the second may reuse the first
// one's freed addresses: the compat layer's weight cache must notice).
// prints one line per forward: "logits <pos> <argmax> <v0> <v1> ... <v_{k-1}>"
// (first min(vocab, 16) logits, %.9g) so a test can compare them with the
// reference CPU path's fixtures.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gguf.h"
#include "model.h"
#include "ops.h"

bool verbose_g = false;  // defined by the program, as main.cpp:11 does (common.h:7)

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s model.gguf n_decode tok0 [tok1 ...]\n", argv[0]);
    return 2;
  }
  try {
    init_ops(0);
    const int n_decode = atoi(argv[2]);
    std::vector<int> prompt;
    for (int i = 3; i < argc; i++) prompt.push_back(atoi(argv[i]));
    std::vector<std::string> paths;
    for (const char *p = argv[1], *q; *p; p = *q ? q + 1 : q) {
      q = p;
      while (*q && *q != ',') q++;
      paths.emplace_back(p, q);
    }
    for (size_t mi = 0; mi < paths.size(); mi++) {
    if (paths.size() > 1) printf("model %zu\n", mi);
    GGUFFile gguf(paths[mi]);
    Model model(gguf);
    auto emit = [](int pos, const std::vector<float>& lg) {
      int am = 0;
      for (size_t i = 1; i < lg.size(); i++)
        if (lg[i] > lg[am]) am = (int)i;  // first maximal index (main.cpp:193-194)
      printf("logits %d %d", pos, am);
      for (size_t i = 0; i < lg.size() && i < 16; i++) printf(" %.9g", lg[i]);
      printf("\n");
      return am;
    };
    auto out = model.forward(prompt, 0);
    int pos = (int)prompt.size();
    int tok = emit(pos - 1, out.back());
    for (int s = 0; s < n_decode; s++) {
      out = model.forward({tok}, pos);
      tok = emit(pos, out.back());
      pos++;
    }
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
