// rccl_sum.cpp — the one collective of the path: a sum of the per-GPU verdict
// histograms (EBPF_HIST_BINS u64) across the GPUs of this process, over RCCL (xGMI).
//
// RCCL is loaded on first use (dlopen of librccl.so.1), so single-GPU users of the library do
// not need it, and a process that already has torch's RCCL (same soname) shares that one copy.
// Communicators are built once per ordered device list (ncclCommInitAll) and kept.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "internal.h"

namespace {

struct rccl_api {
	bool loaded = false;
	std::string err;
	ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
	ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t,
				   ncclComm_t, hipStream_t) = nullptr;
	ncclResult_t (*group_start)() = nullptr;
	ncclResult_t (*group_end)() = nullptr;
	const char *(*error_string)(ncclResult_t) = nullptr;
};

std::mutex g_lock;
rccl_api g_api;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

template <class F>
bool
sym(void *h, const char *name, F *out)
{
	*out = reinterpret_cast<F>(dlsym(h, name));
	return *out != nullptr;
}

// under g_lock
bool
load()
{
	if (g_api.loaded)
		return true;
	if (!g_api.err.empty())
		return false;
	void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
	if (!h)
		h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
	if (!h) {
		g_api.err = std::string("cannot load RCCL: ") + dlerror();
		return false;
	}
	if (!sym(h, "ncclCommInitAll", &g_api.comm_init_all) ||
	    !sym(h, "ncclAllReduce", &g_api.all_reduce) || !sym(h, "ncclGroupStart", &g_api.group_start) ||
	    !sym(h, "ncclGroupEnd", &g_api.group_end) ||
	    !sym(h, "ncclGetErrorString", &g_api.error_string)) {
		g_api.err = "RCCL lacks a required symbol";
		return false;
	}
	g_api.loaded = true;
	return true;
}

} // namespace

// Sum hist[d] (EBPF_HIST_BINS u64 on devices[d], distinct devices) over d in place, each on
// streams[d], as one RCCL group.  Asynchronous.  hist[d] is the library's scratch, never a caller's
// histogram (ebpf_prog_run_batch_multi_dev adds the sum into those afterwards).  Returns 0, ENOSYS (no RCCL) or EIO (RCCL error; *msg says which).
int
rccl_hist_allreduce(int ndev, const int *devices, uint64_t *const *hist, hipStream_t *streams,
		    std::string *msg)
{
	std::lock_guard<std::mutex> g(g_lock);
	device_guard dg;
	if (!load()) {
		*msg = g_api.err;
		return ENOSYS;
	}
	std::vector<int> key(devices, devices + ndev);
	auto it = g_comms.find(key);
	if (it == g_comms.end()) {
		std::vector<ncclComm_t> comms(ndev);
		ncclResult_t r = g_api.comm_init_all(comms.data(), ndev, devices);
		if (r != ncclSuccess) {
			*msg = std::string("ncclCommInitAll: ") + g_api.error_string(r);
			return EIO;
		}
		it = g_comms.emplace(key, std::move(comms)).first;
	}
	ncclResult_t r = g_api.group_start();
	for (int d = 0; d < ndev && r == ncclSuccess; d++) {
		if (hipSetDevice(devices[d]) != hipSuccess) {
			g_api.group_end();
			*msg = "hipSetDevice";
			return EIO;
		}
		r = g_api.all_reduce(hist[d], hist[d], EBPF_HIST_BINS, ncclUint64, ncclSum, it->second[d],
				     streams[d]);
	}
	ncclResult_t r2 = g_api.group_end();
	if (r == ncclSuccess)
		r = r2;
	if (r != ncclSuccess) {
		*msg = std::string("ncclAllReduce: ") + g_api.error_string(r);
		return EIO;
	}
	return 0;
}
