// async.cpp — the host-buffer batch without blocking the caller (a NIC-ring
// or capture consumer fills its next segment while the GPU works on this one).  A job runs the
// same pipeline as ebpf_prog_run_batch (chunked H2D -> kernel -> D2H on the library's streams)
// on a worker bound to the caller's current device; the caller collects it with ebpf_batch_wait.
//
// Per device there is a persistent pool of kWorkers threads (started on the first job, kept for
// the life of the process) fed by a bounded FIFO of kQueueDepth jobs: two workers keep one job's
// copies overlapping the next one's, and a consumer that submits faster than PCIe drains gets
// EAGAIN instead of an unbounded pile of threads.  Jobs on one device share its staging pool.
#include <cerrno>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"

struct ebpf_batch_job {
	struct ebpf_prog *ep = nullptr;
	ebpf_pkt_batch batch;   // the caller's descriptor, copied (its buffers stay the caller's)
	uint64_t *ret = nullptr;
	uint8_t *faults = nullptr;
	ebpf_batch_stats stats;
	int rc = 0;
	std::string msg;
	std::mutex m;
	std::condition_variable cv;
	bool done = false;
};

namespace {

constexpr int kWorkers = 2;
constexpr size_t kQueueDepth = 64; // jobs queued (not yet started) per device

struct device_pool {
	int device = 0;
	std::mutex m;
	std::condition_variable cv;
	std::deque<ebpf_batch_job *> q;
	bool started = false;
};

std::mutex g_pools_lock;
std::vector<device_pool *> g_pools; // per device; never freed (its workers live until exit)

void
worker(device_pool *P)
{
	ebpf_gpu_set_device(P->device);
	for (;;) {
		ebpf_batch_job *j;
		{
			std::unique_lock<std::mutex> g(P->m);
			P->cv.wait(g, [P] { return !P->q.empty(); });
			j = P->q.front();
			P->q.pop_front();
		}
		j->rc = ebpf_prog_run_batch(j->ep, &j->batch, j->ret, j->faults, &j->stats);
		if (j->rc)
			j->msg = ebpf_gpu_last_error();
		// (notified under the lock: once it is released the waiter may free the job)
		std::lock_guard<std::mutex> g(j->m);
		j->done = true;
		j->cv.notify_all();
	}
}

// The device's pool, its workers started (0), or EAGAIN when no thread could be created.
int
pool_for(int device, device_pool **out)
{
	std::lock_guard<std::mutex> g(g_pools_lock);
	if ((int)g_pools.size() <= device)
		g_pools.resize(device + 1, nullptr);
	if (g_pools[device] == nullptr) {
		g_pools[device] = new (std::nothrow) device_pool;
		if (g_pools[device] == nullptr)
			return ENOMEM;
		g_pools[device]->device = device;
	}
	device_pool *P = g_pools[device];
	if (!P->started) {
		try {
			for (int w = 0; w < kWorkers; w++)
				std::thread(worker, P).detach();
		} catch (...) {
			return EAGAIN; // (threads already started keep serving the queue)
		}
		P->started = true;
	}
	*out = P;
	return 0;
}

} // namespace

EBPF_EXPORT int
ebpf_prog_run_batch_async(struct ebpf_prog *ep, const struct ebpf_pkt_batch *batch, uint64_t *ret,
			  uint8_t *faults, struct ebpf_batch_job **job)
{
	if (job == nullptr || ep == nullptr || batch == nullptr || ret == nullptr) {
		set_last_error("prog, batch, ret or job is NULL");
		return EINVAL;
	}
	*job = nullptr;
	if (ebpf_gpu_device_count() == 0) {
		set_last_error("no GPU visible");
		return ENODEV;
	}
	device_pool *P;
	int err = pool_for(current_device(), &P);
	if (err) {
		set_last_error("no worker thread for the device");
		return err;
	}
	ebpf_batch_job *j = new (std::nothrow) ebpf_batch_job;
	if (j == nullptr)
		return ENOMEM;
	j->ep = ep;
	j->batch = *batch;
	j->ret = ret;
	j->faults = faults;
	{
		std::lock_guard<std::mutex> g(P->m);
		if (P->q.size() >= kQueueDepth) {
			delete j;
			set_last_error("the device's job queue is full (wait for earlier jobs)");
			return EAGAIN;
		}
		P->q.push_back(j);
	}
	P->cv.notify_one();
	*job = j;
	return 0;
}

EBPF_EXPORT int
ebpf_batch_wait(struct ebpf_batch_job *job, struct ebpf_batch_stats *stats)
{
	if (job == nullptr) {
		set_last_error("job is NULL");
		return EINVAL;
	}
	{
		std::unique_lock<std::mutex> g(job->m);
		job->cv.wait(g, [job] { return job->done; });
	}
	const int rc = job->rc;
	if (rc)
		set_last_error(job->msg);
	else if (stats)
		*stats = job->stats;
	delete job;
	return rc;
}
