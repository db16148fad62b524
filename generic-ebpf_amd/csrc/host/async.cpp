// async.cpp — the host-buffer batch without blocking the caller (a NIC-ring
// or capture consumer fills its next segment while the GPU works on this one).  A job runs the
// same pipeline as ebpf_prog_run_batch (chunked H2D -> kernel -> D2H on the library's streams)
// on a worker bound to the caller's current device; the caller collects it with ebpf_batch_wait.
//
// Per device there is a persistent pool of kWorkers threads (started on the first job, kept for
// the life of the process) fed by a bounded FIFO of kQueueDepth jobs: two workers keep one job's
// copies overlapping the next one's, and a consumer that submits faster than PCIe drains gets
// EAGAIN instead of an unbounded pile of threads.  Jobs on one device share its staging pool.
//
// Two properties of ebpf_prog_run_batch that a worker thread would otherwise lose:
//   * percpu maps index the CPU the batch is submitted from (map_current_cpu: the first CPU of the
//     calling thread's affinity mask, ebpf_linux_user.c:83-112).  A job carries its submitter's
//     mask and the worker runs it under that mask;
//   * jobs of map-writing programs behave as if run one after the other in submission order (each
//     batch reads what the earlier ones wrote; ebpf_gpu.h "Map writes in a device batch"): such a
//     job takes a ticket when it is queued, and a worker runs it only when every writing job with
//     an earlier ticket has finished, on whichever device it was queued.
#include <pthread.h>
#include <sched.h>

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
	cpu_set_t affinity;      // the submitting thread's CPU mask
	bool has_affinity = false;
	uint64_t writer = 0;     // map-writing program: its ticket (1, 2, ...), else 0
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
	int nworkers = 0; // workers running (kWorkers once every start succeeded)
};

std::mutex g_pools_lock;
std::vector<device_pool *> g_pools; // per device; never freed (its workers live until exit)

// Tickets of map-writing jobs, across devices: the next one to hand out, the next one to run.
// (A queue is FIFO and a ticket is taken as the job is queued, so the earliest unfinished writer
// is at its queue's front once the jobs ahead of it are done: waiting for it cannot deadlock.)
std::mutex g_writers_lock;
std::condition_variable g_writers_cv;
uint64_t g_writer_next_ticket = 1, g_writer_next_run = 1;

bool
writes_maps(struct ebpf_prog *ep)
{
	if (prog_ensure_translated(ep) != 0)
		return false; // (the job fails with the same error when it runs)
	return prog_writes_maps(*ep->xlated);
}

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
		if (j->has_affinity)
			pthread_setaffinity_np(pthread_self(), sizeof(j->affinity), &j->affinity);
		if (j->writer) {
			std::unique_lock<std::mutex> g(g_writers_lock);
			g_writers_cv.wait(g, [j] { return g_writer_next_run == j->writer; });
		}
		j->rc = ebpf_prog_run_batch(j->ep, &j->batch, j->ret, j->faults, &j->stats);
		if (j->rc)
			j->msg = ebpf_gpu_last_error();
		if (j->writer) {
			std::lock_guard<std::mutex> g(g_writers_lock);
			g_writer_next_run++;
			g_writers_cv.notify_all();
		}
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
	// top the pool up to kWorkers (a start that failed earlier is retried; the threads that
	// did start keep serving the queue)
	while (P->nworkers < kWorkers) {
		try {
			std::thread(worker, P).detach();
		} catch (...) {
			break;
		}
		P->nworkers++;
	}
	if (P->nworkers == 0)
		return EAGAIN;
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
	j->has_affinity = pthread_getaffinity_np(pthread_self(), sizeof(j->affinity), &j->affinity) == 0;
	const bool writer = writes_maps(ep);
	{
		std::lock_guard<std::mutex> g(P->m);
		if (P->q.size() >= kQueueDepth) {
			delete j;
			set_last_error("the device's job queue is full (wait for earlier jobs)");
			return EAGAIN;
		}
		if (writer) { // (taken with the queue slot: a ticket is never left unused)
			std::lock_guard<std::mutex> w(g_writers_lock);
			j->writer = g_writer_next_ticket++;
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
