// main_mi355x.cpp -- the reference's greedy decode loop (main.cpp:160-224)
// with the forward pass served by the MI355X device session of libllmi.so.
//
// The reference's own GGUFFile / Model (gguf.cpp, model.cpp, compiled
// unchanged) parse the file and tokenize the prompt exactly as main.cpp does
// (main.cpp:70-140); every forward goes through include/llmi.h instead of
// Model::forward.  Two loop shapes:
//   default        main.cpp's loop as written: llmi_session_forward for the
//                  prompt (batched prefill on the device), then one
//                  llmi_session_forward per generated token, greedy argmax of
//                  the returned logits on the host (std::max_element,
//                  main.cpp:193-194), EOS / end-of-turn stop (main.cpp:196-198);
//   --device-loop  the same tokens from llmi_session_generate: the argmax is
//                  fed back on the device, one hipGraph replay per token, no
//                  host round trip; the ids are then printed up to the first
//                  EOS / end-of-turn like the host loop.
// Usage:
//   main_mi355x -m model.gguf [-p prompt | --tokens "2 17 301"] [-n 100]
//               [--no-cnv] [--exact] [--device-loop]
// Output: the generated text (token strings), then "ids: ..." and main.cpp's
// "Generated N tokens in T s (X tok/s)" line.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "gguf.h"
#include "llmi.h"
#include "model.h"
#include "ops.h"

bool verbose_g = false;  // main.cpp:11

static std::string replace_special_space(const std::string& token) {  // main.cpp:15-26 (same behaviour)
  static const std::string sp = u8"▁";
  std::string r = token;
  for (size_t p = 0; (p = r.find(sp, p)) != std::string::npos; p += 1) r.replace(p, sp.size(), " ");
  return r;
}

static void check(int rc, const char* what) {
  if (rc != LLMI_OK) throw std::runtime_error(std::string(what) + ": " + llmi_last_error());
}

int main(int argc, char** argv) {
  std::string model_path, prompt = "One sentence fact about silicon", tok_list;
  int n_predict = 100;
  bool chat = true, exact = false, device_loop = false;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value after " + a);
      return argv[++i];
    };
    if (a == "-m" || a == "--model") model_path = next();
    else if (a == "-p" || a == "--prompt") prompt = next();
    else if (a == "-n" || a == "--predict") n_predict = std::stoi(next());
    else if (a == "-t" || a == "--threads") next();  // host threads: unused (the forward runs on the GPU)
    else if (a == "--no-cnv") chat = false;
    else if (a == "--exact") exact = true;
    else if (a == "--device-loop") device_loop = true;
    else if (a == "--tokens") tok_list = next();
    else if (a == "-v" || a == "--verbose") verbose_g = true;
    else {
      std::cerr << "unknown option " << a << "\n";
      return 2;
    }
  }
  if (model_path.empty()) {
    std::cerr << "Error: Model file not specified." << std::endl;  // main.cpp:64-67
    return 1;
  }
  try {
    init_ops(1);  // the reference's pool (tokenization does not use it)
    GGUFFile gguf_file(model_path);
    Model model(gguf_file);  // for tokenize() only: the forward runs on the device
    std::vector<int> tokens;
    if (!tok_list.empty()) {
      std::istringstream is(tok_list);
      for (int t; is >> t;) tokens.push_back(t);
    } else {
      bool prefilled_thinking = false;
      tokens = model.tokenize(prompt, chat, &prefilled_thinking);  // main.cpp:107-109
    }
    const auto& metadata = gguf_file.get_metadata();  // main.cpp:118-137
    std::vector<std::string> token_strings;
    for (const auto& t : metadata.at("tokenizer.ggml.tokens").arr) token_strings.push_back(t.str);
    int end_of_turn_token_id = -1;
    for (size_t i = 0; i < token_strings.size(); ++i)
      if (token_strings[i] == "<end_of_turn>" || token_strings[i] == "<turn|>") {
        end_of_turn_token_id = (int)i;
        break;
      }
    int eos_token_id = -1;
    if (metadata.count("tokenizer.ggml.eos_token_id"))
      eos_token_id = (int)metadata.at("tokenizer.ggml.eos_token_id").scalar.u32;

    // the device session reads the same file bytes (mapped read-only)
    const int fd = open(model_path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + model_path);
    struct stat st;
    fstat(fd, &st);
    void* map = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (map == MAP_FAILED) throw std::runtime_error("cannot map " + model_path);
    llmi_session_opts opts{};
    opts.flags = exact ? LLMI_EXACT : 0u;
    opts.max_ctx = (int)tokens.size() + n_predict + 8;
    opts.tp_size = 1;
    llmi_session* sess = nullptr;
    check(llmi_session_create(map, (size_t)st.st_size, &opts, &sess), "llmi_session_create");
    munmap(map, (size_t)st.st_size);  // the session uploaded everything it needs
    llmi_session_info info{};
    check(llmi_session_get_info(sess, &info), "llmi_session_get_info");

    std::cout << "Prompt: " << prompt << "\n\n";
    std::vector<float> logits((size_t)info.vocab);
    int32_t first = 0;
    // prompt: model.forward(tokens, 0) (main.cpp:163)
    check(llmi_session_forward(sess, tokens.data(), (int)tokens.size(), 0, logits.data(), &first), "forward");
    int pos = (int)tokens.size();
    std::vector<int> ids;
    const auto start_time = std::chrono::high_resolution_clock::now();
    int num_generated_tokens = 0;
    auto emit = [&](int next_token) -> bool {  // false: stop (main.cpp:196-198)
      if (next_token == end_of_turn_token_id || next_token == eos_token_id) return false;
      ids.push_back(next_token);
      std::cout << replace_special_space(token_strings[(size_t)next_token]);
      std::cout.flush();
      num_generated_tokens++;
      return true;
    };
    if (!device_loop) {
      for (int i = 0; i < n_predict; ++i) {
        const int next_token =
            (int)std::distance(logits.begin(), std::max_element(logits.begin(), logits.end()));  // main.cpp:193-194
        if (!emit(next_token)) break;
        if (i < n_predict - 1) {  // model.forward({next_token}, pos) (main.cpp:218-223)
          int32_t t = next_token;
          check(llmi_session_forward(sess, &t, 1, pos, logits.data(), nullptr), "forward");
          pos++;
        }
      }
    } else if (n_predict > 0) {
      // argmax of the prompt's logits, then n_predict - 1 device steps
      std::vector<int32_t> out((size_t)std::max(1, n_predict - 1));
      if (n_predict > 1) check(llmi_session_generate(sess, first, pos, n_predict - 1, out.data()), "generate");
      std::vector<int> all{first};
      all.insert(all.end(), out.begin(), out.begin() + (n_predict - 1));
      for (int t : all)
        if (!emit(t)) break;
    }
    const auto end_time = std::chrono::high_resolution_clock::now();
    const double el = std::chrono::duration<double>(end_time - start_time).count();
    std::cout << std::endl << "ids:";
    for (int t : ids) std::cout << " " << t;
    std::cout << std::endl;
    std::cout << "\nGenerated " << num_generated_tokens << " tokens in " << el << " s ("
              << num_generated_tokens / el << " tok/s)" << std::endl;  // main.cpp:226-232
    llmi_session_destroy(sess);
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
