// tpe_pool.h — the host runtime's worker pool (tpe_pool.cpp), internal.
//
// The per-label host work of a suggest (the Parzen fits of every label a tree
// level needs, tpe.py:398-475 / 573-607 per label) is independent across
// labels; the reference does it one label at a time inside its pyll
// interpreter.  parallel_for runs such per-label jobs on a few resident worker
// threads plus the caller, so the host part of a suggest takes as long as its
// slowest label instead of the sum over labels.
#pragma once
#include <cstdint>

namespace tpe_pool {

// fn(ctx, i) for i in [0, n), on the caller and the pool's workers; returns
// when every call has returned.  Serial when the pool is off (tpe_host_threads
// 0), when n < 2, or when another thread holds the pool (nested or concurrent
// callers never wait on each other).
void parallel_for(int n, void (*fn)(void* ctx, int i), void* ctx);

// workers the next parallel_for may use (the caller not counted)
int workers();

}  // namespace tpe_pool

// tpe_host_pack_level's early hook (internal, per thread): tpe_level_run sets it
// around its pack; the packer calls fn once the blob's leading sections are
// placed and its device-fit jobs written, before the fill — `early` holds the
// leading offsets, the fit counts, the bytes to upload (up_off / up_len[0]) and
// the device bytes the fit touches (blob_bytes) — so the device fit can run
// while the host fills the rest.  {nullptr, nullptr}: no hook.
struct tpe_pack_info;
struct TpePackHook {
  void (*fn)(void* ctx, const struct tpe_pack_info* early);
  void* ctx;
};
extern "C" void tpe_internal_pack_hook(TpePackHook h);
