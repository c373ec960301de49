// SlotGroupCommit (csrc/engine.h) with carried requests, host only: callers
// on threads post requests of 1-3 pieces; the batched call advances every
// stream of its batch by one piece and leaves unfinished requests to the next
// batch.  Checks: a caller returns only when its request is complete, every
// piece runs exactly once and in order, a batch holds a stream at most once,
// and an unfinished request leads the next batch.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "engine.h"

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 8, N = argc > 2 ? atoi(argv[2]) : 300;
  vamd::SlotGroupCommit gc;
  gc.Resize(S);
  gc.SetWindowUs(200);
  struct Req {
    int id = -1, pieces = 0, done = 0;
  };
  std::vector<Req> cur(S);
  std::vector<std::vector<std::pair<int, int>>> log(S);  // (request, piece) as run
  std::vector<int> carried;                                // unfinished streams of the last batch
  int bad = 0;
  std::mutex mu;
  auto batch_fn = [&](const std::vector<int>& batch, std::vector<char>* complete) {
    std::lock_guard<std::mutex> lk(mu);  // (one leader at a time; the lock only guards the checks)
    std::vector<char> seen(S, 0);
    for (size_t i = 0; i < batch.size(); i++) {
      const int s = batch[i];
      if (seen[s]++) bad |= 1;  // a stream twice in one batch
      if (i < carried.size() && carried[i] != s) bad |= 2;  // carried requests lead, in order
    }
    if (batch.size() < carried.size()) bad |= 2;
    carried.clear();
    for (size_t i = 0; i < batch.size(); i++) {
      Req& r = cur[batch[i]];
      log[batch[i]].push_back({r.id, r.done});
      r.done++;
      (*complete)[i] = r.done >= r.pieces;
      if (!(*complete)[i]) carried.push_back(batch[i]);
    }
  };
  std::vector<std::thread> th;
  for (int s = 0; s < S; s++)
    th.emplace_back([&, s] {
      std::mt19937 rng(1234 + s);
      for (int n = 0; n < N; n++) {
        {
          std::lock_guard<std::mutex> lk(mu);
          cur[s].id = n;
          cur[s].pieces = 1 + (int)(rng() % 3);
          cur[s].done = 0;
        }
        gc.Run(s, batch_fn);
        std::lock_guard<std::mutex> lk(mu);
        if (cur[s].done != cur[s].pieces) bad |= 4;  // returned before its request was complete
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
      }
    });
  for (auto& t : th) t.join();
  long long pieces = 0;
  for (int s = 0; s < S; s++) {
    std::mt19937 rng(1234 + s);
    size_t k = 0;
    for (int n = 0; n < N; n++) {
      const int np = 1 + (int)(rng() % 3);
      if (rng() % 4 == 0) (void)rng();
      for (int p = 0; p < np; p++, k++)
        if (k >= log[s].size() || log[s][k] != std::make_pair(n, p)) bad |= 8;  // every piece once, in order
    }
    if (k != log[s].size()) bad |= 8;
    pieces += (long long)log[s].size();
  }
  printf("streams %d requests %d pieces %lld bad %d\n", S, N, pieces, bad);
  return bad ? 1 : 0;
}
