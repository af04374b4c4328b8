//go:build linux && cgo

// Package gpu serves Weaviate's VectorIndex search path from libwvgpu.so, the
// MI355X engine of this repository, behind the reference's own interface
// (adapters/repos/db/vector_index.go:23-40).  It is the file a maintainer
// commits as adapters/repos/db/vector/gpu/gpu.go; the factory change in
// adapters/repos/db/shard.go:134-172 is shown in INTEGRATION.md.
//
// The decorator wraps the shard's CPU hnsw index.  The CPU index keeps
// persistence (commit log, snapshots), maintenance and every write; each
// write is then propagated to a GPU mirror (wv_mirror_* in include/wvgpu.h),
// whose whole lifecycle lives in the library so that the native replay
// harness (tests/native/mirror_replay.cpp) tests exactly the calls below:
//
//	New              -> wv_mirror_create (dims learnt lazily, insert.go:43-65)
//	PostStartup      -> cpu.PostStartup, a log flush, then
//	                    wv_mirror_post_startup_async: on the library's own
//	                    thread the shard's commit log
//	                    <RootPath>/<ID>.hnsw.commitlog.d is replayed as
//	                    restoreFromDisk does (startup.go:56-152) and the rows
//	                    are pulled through VectorForIDThunk (shard.go:165),
//	                    while the CPU index serves (the reference prefills its
//	                    cache in a goroutine, startup.go:174-203); writes that
//	                    arrive meanwhile are replayed when it goes live
//	Add(id, vec)     -> cpu.Add, then wv_mirror_add (the mirror grows like
//	                    growIndexToAccomodateNode, maintainance.go:69-100)
//	Delete(ids...)   -> cpu.Delete, then wv_mirror_delete (delete.go:29-84)
//	SearchByVector   -> wv_mirror_search (micro-batched; search.go:64-79)
//	SearchByVectorDistance -> wv_mirror_search_by_distance (search.go:90-158)
//	UpdateUserConfig -> cpu.UpdateUserConfig, then wv_mirror_update_config;
//	                    PQ enabled at runtime: the CPU index answers until a
//	                    flush + wv_mirror_compact after Compress turned the
//	                    mirror to the codes (config_update.go:97-120)
//
// Rows added after the last graph snapshot are searched exactly beside the
// graph; once wv_mirror_needs_compaction reports enough of them, a background
// goroutine flushes the CPU index's commit log (hnsw.Flush, index.go:650-652)
// and calls wv_mirror_compact, which re-snapshots the mirror's graph from the
// log -- the CPU index's own graph.
//
// A write the mirror cannot take marks it stale (the library refuses reads
// with WV_ESTALE): searches are then answered by the CPU index, so a stale
// mirror never serves a deleted id or misses an added one, and the library
// resyncs it in the background (wvgpuFlush flushes the CPU index's log first,
// then the startup runs again; 1 s doubling to 60 s between failed tries).
// Writes hold mu shared across the CPU write and its propagation; compaction
// and the resync's flush hold it exclusively while they flush the log, so
// every node the flushed log holds has reached the mirror.  PQ-compressed
// classes (KMeans encoder) are served compressed from the log's quantizer.
//
// The Go toolchain is not part of the image this engine is developed in, so
// this file has not been type-checked; tests/native/mirror_replay.cpp
// replays its C call sequence against the library on the GPU.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../weaviate_amd -lwvgpu -Wl,-rpath,${SRCDIR}/../../../weaviate_amd
#include <stdlib.h>
#include "wvgpu.h"

// the exported Go thunks (below), as a wv_vector_source and a wv_flush_fn
extern int wvgpuVectorForID(void *ctx, uint64_t id, float *out, int cap, int *len);
extern int wvgpuFlush(void *ctx);
static int wvgpu_post_startup_async(wv_mirror *m, void *ctx) {
	return wv_mirror_post_startup_async(m, wvgpuVectorForID, ctx);
}
static void wvgpu_self_heal(wv_mirror_options *o, void *ctx) {
	o->auto_resync = 1;
	o->flush = wvgpuFlush;
	o->flush_ctx = ctx;
}
*/
import "C"

import (
	"context"
	"runtime/cgo"
	"sync"
	"sync/atomic"
	"time"
	"unsafe"

	"github.com/pkg/errors"
	"github.com/weaviate/weaviate/adapters/repos/db/helpers"
	"github.com/weaviate/weaviate/entities/schema"
	"github.com/weaviate/weaviate/entities/storobj"
	ent "github.com/weaviate/weaviate/entities/vectorindex/hnsw"
)

// cpuIndex is the VectorIndex the decorator wraps (vector_index.go:23-40).
type cpuIndex interface {
	Dump(labels ...string)
	Add(id uint64, vector []float32) error
	Delete(id ...uint64) error
	SearchByVector(vector []float32, k int, allow helpers.AllowList) ([]uint64, []float32, error)
	SearchByVectorDistance(vector []float32, dist float32, maxLimit int64,
		allow helpers.AllowList) ([]uint64, []float32, error)
	UpdateUserConfig(updated schema.VectorIndexConfig, callback func()) error
	Drop(ctx context.Context) error
	Shutdown(ctx context.Context) error
	Flush() error
	PauseMaintenance(ctx context.Context) error
	SwitchCommitLogs(ctx context.Context) error
	ListFiles(ctx context.Context) ([]string, error)
	ResumeMaintenance(ctx context.Context) error
	PostStartup()
	ValidateBeforeInsert(vector []float32) error
}

// VectorForID is hnsw.VectorForID (hnsw/index.go): the shard's
// vectorByIndexID (shard_read.go:145-161).
type VectorForID func(ctx context.Context, id uint64) ([]float32, error)

// Metric values of wv_metric (distancer.Provider.Type(), provider.go:14-24).
const (
	MetricL2Squared = C.WV_L2_SQUARED
	MetricDot       = C.WV_DOT
	MetricCosineDot = C.WV_COSINE_DOT
)

// Index is a VectorIndex whose searches run on one MI355X.
type Index struct {
	cpuIndex
	m          *C.wv_mirror
	logDir     *C.char
	vectorFor  VectorForID
	device     int
	mu         sync.RWMutex // calls shared; the log flushes, PostStartup and close exclusive
	compacting atomic.Bool
	closed     atomic.Bool
	pqPending  atomic.Bool // PQ enabled at runtime, the mirror not yet serving the codes: the CPU index answers
	pqGen      atomic.Int64 // one per runtime PQ enablement (its callbacks count against it)
	pqCalls    atomic.Int32 // callbacks seen for the current pqGen: the second one follows Compress's end
	handle     cgo.Handle      // this Index, for the library's callbacks (its threads call them)
	ctx        *C.uintptr_t    // C memory holding handle: the callbacks' ctx, valid until close
	metrics    *mirrorMetrics  // nil unless Options.Metrics
}

// Options: the shard's paths and the mirror's sizes.
type Options struct {
	Device       int
	RootPath     string      // hnsw.Config.RootPath
	ID           string      // hnsw.Config.ID: the log is RootPath/ID.hnsw.commitlog.d
	VectorForID  VectorForID // hnsw.Config.VectorForIDThunk
	MaxBatch     int         // queries per coalesced launch (0: 1024)
	MaxWaitUsec  int         // micro-batcher linger at an idle device (0: none, launch at once)
	CompactRows  uint64      // delta rows that trigger a compaction (0: 8192)
	InitialSize  uint64      // mirror capacity before growth (0: 25000)
	Metrics      bool        // export the mirror's gauges (metrics.go; PROMETHEUS_MONITORING_ENABLED)
	ClassName    string      // metric labels, as hnsw's Metrics (metrics.go:23-228)
	ShardName    string
}

func lastErr(op string, rc C.int) error {
	return errors.Errorf("wvgpu %s: status %d: %s", op, int(rc), C.GoString(C.wv_last_error()))
}

func configOf(uc ent.UserConfig, device int) C.wv_config {
	var cfg C.wv_config
	C.wv_config_default(&cfg)
	cfg.device = C.int(device)
	cfg.max_connections = C.int(uc.MaxConnections)
	cfg.ef = C.int64_t(uc.EF)
	cfg.dynamic_ef_min = C.int64_t(uc.DynamicEFMin)
	cfg.dynamic_ef_max = C.int64_t(uc.DynamicEFMax)
	cfg.dynamic_ef_factor = C.int64_t(uc.DynamicEFFactor)
	cfg.flat_search_cutoff = C.int64_t(uc.FlatSearchCutoff)
	return cfg
}

// New creates the mirror.  It serves searches after PostStartup.
func New(cpu cpuIndex, metric int, uc ent.UserConfig, opt Options) (*Index, error) {
	if opt.VectorForID == nil || opt.RootPath == "" || opt.ID == "" {
		return nil, errors.New("wvgpu: RootPath, ID and VectorForID are required")
	}
	cfg := configOf(uc, opt.Device)
	g := &Index{cpuIndex: cpu, vectorFor: opt.VectorForID, device: opt.Device}
	g.logDir = C.CString(opt.RootPath + "/" + opt.ID + ".hnsw.commitlog.d")
	g.handle = cgo.NewHandle(g)
	g.ctx = (*C.uintptr_t)(C.malloc(C.size_t(unsafe.Sizeof(C.uintptr_t(0)))))
	*g.ctx = C.uintptr_t(g.handle)
	var mo C.wv_mirror_options
	mo.initial_capacity = C.uint64_t(opt.InitialSize)
	mo.max_batch = C.int(opt.MaxBatch)
	mo.max_wait_us = C.int(opt.MaxWaitUsec)
	mo.compact_rows = C.uint64_t(opt.CompactRows)
	mo.commitlog_dir = g.logDir
	C.wvgpu_self_heal(&mo, unsafe.Pointer(g.ctx))
	if rc := C.wv_mirror_create(C.int(metric), &cfg, &mo, &g.m); rc != 0 {
		g.freeHandles()
		return nil, lastErr("create", rc)
	}
	if opt.Metrics {
		g.metrics = newMirrorMetrics(g, opt.ClassName, opt.ShardName)
	}
	return g, nil
}

func (g *Index) freeHandles() {
	C.free(unsafe.Pointer(g.logDir))
	C.free(unsafe.Pointer(g.ctx))
	g.handle.Delete()
}

//export wvgpuFlush
func wvgpuFlush(ctx unsafe.Pointer) C.int {
	g := cgo.Handle(*(*C.uintptr_t)(ctx)).Value().(*Index)
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.closed.Load() {
		return C.WV_ESTATE
	}
	if err := g.cpuIndex.Flush(); err != nil {
		return C.WV_ESTATE
	}
	return C.WV_OK
}

//export wvgpuVectorForID
func wvgpuVectorForID(ctx unsafe.Pointer, id C.uint64_t, out *C.float, capacity C.int, length *C.int) C.int {
	g := cgo.Handle(*(*C.uintptr_t)(ctx)).Value().(*Index)
	vec, err := g.vectorFor(context.Background(), uint64(id))
	if err != nil {
		var nf storobj.ErrNotFound
		if errors.As(err, &nf) {
			return C.WV_ENOTFOUND // search.go's handleDeletedNode path
		}
		return C.WV_EINVAL
	}
	*length = C.int(len(vec))
	if len(vec) > 0 && len(vec) <= int(capacity) {
		dst := unsafe.Slice((*float32)(unsafe.Pointer(out)), len(vec))
		copy(dst, vec)
	}
	return C.WV_OK
}

// PostStartup: the CPU index's own routines, then the mirror loads from the
// shard's commit log and object store on the library's thread
// (startup.go:169-205); the CPU index serves until it is live.
func (g *Index) PostStartup() {
	g.cpuIndex.PostStartup()
	g.mu.Lock() // every write before the flush is in the log, every later one is replayed
	defer g.mu.Unlock()
	if g.closed.Load() {
		return
	}
	if err := g.cpuIndex.Flush(); err != nil {
		return // the mirror stays idle: the CPU index serves
	}
	C.wvgpu_post_startup_async(g.m, unsafe.Pointer(g.ctx))
}

// Add mirrors hnsw.Add (insert.go:43-65).
func (g *Index) Add(id uint64, vector []float32) error {
	g.mu.RLock()
	if err := g.cpuIndex.Add(id, vector); err != nil {
		g.mu.RUnlock()
		return err
	}
	compact := false
	if !g.closed.Load() {
		if len(vector) > 0 {
			C.wv_mirror_add(g.m, C.uint64_t(id), (*C.float)(unsafe.Pointer(&vector[0])), C.int(len(vector)))
		}
		compact = C.wv_mirror_needs_compaction(g.m) != 0 // (under mu: close cannot free the mirror meanwhile)
	}
	g.mu.RUnlock()
	if compact {
		g.startCompaction()
	}
	return nil
}

// Delete mirrors hnsw.Delete (delete.go:29-84): tombstones reach the mirror
// before Delete returns.
func (g *Index) Delete(ids ...uint64) error {
	g.mu.RLock()
	defer g.mu.RUnlock()
	if err := g.cpuIndex.Delete(ids...); err != nil || g.closed.Load() {
		return err
	}
	if len(ids) > 0 {
		C.wv_mirror_delete(g.m, (*C.uint64_t)(unsafe.Pointer(&ids[0])), C.uint64_t(len(ids)))
	}
	return nil
}

// startCompaction re-snapshots the mirror's graph from the flushed commit
// log once the delta has grown past Options.CompactRows.
func (g *Index) startCompaction() {
	if !g.compacting.CompareAndSwap(false, true) {
		return
	}
	go func() {
		defer g.compacting.Store(false)
		g.mu.Lock()
		if g.closed.Load() {
			g.mu.Unlock()
			return
		}
		err := g.cpuIndex.Flush()
		g.mu.Unlock()
		g.mu.RLock() // (close waits for it)
		if err == nil && !g.closed.Load() {
			C.wv_mirror_compact(g.m) // the log is read without blocking searches
		}
		g.mu.RUnlock()
	}()
}

func allowIDs(allow helpers.AllowList) (*C.uint64_t, C.uint64_t, C.int) {
	if allow == nil {
		return nil, 0, 0
	}
	ids := allow.Slice() // ascending (sroar bitmap)
	if len(ids) == 0 {
		return nil, 0, 1
	}
	return (*C.uint64_t)(unsafe.Pointer(&ids[0])), C.uint64_t(len(ids)), 1
}

// SearchByVector replaces hnsw.SearchByVector (search.go:64-79).
func (g *Index) SearchByVector(vector []float32, k int, allow helpers.AllowList) ([]uint64, []float32, error) {
	g.mu.RLock()
	defer g.mu.RUnlock()
	if len(vector) == 0 || k <= 0 || g.closed.Load() || g.pqPending.Load() {
		return g.cpuIndex.SearchByVector(vector, k, allow)
	}
	ids := make([]uint64, k)
	dists := make([]float32, k)
	var n C.int32_t
	ap, an, filtered := allowIDs(allow)
	rc := C.wv_mirror_search(g.m, (*C.float)(unsafe.Pointer(&vector[0])), C.int(len(vector)), C.int(k), filtered,
		ap, an, (*C.uint64_t)(unsafe.Pointer(&ids[0])), (*C.float)(unsafe.Pointer(&dists[0])), &n)
	switch {
	case rc == C.WV_EDELETED:
		return nil, nil, errors.New("entrypoint was deleted in the object store, " +
			"it has been flagged for cleanup and should be fixed in the next cleanup cycle")
	case rc != 0: // stale mirror or device error: the CPU index answers
		return g.cpuIndex.SearchByVector(vector, k, allow)
	case n == 0:
		return nil, nil, nil // empty index: search.go:463-465
	}
	return ids[:n], dists[:n], nil
}

// SearchByVectorDistance replaces hnsw.SearchByVectorDistance (search.go:90-158).
func (g *Index) SearchByVectorDistance(vector []float32, dist float32, maxLimit int64,
	allow helpers.AllowList,
) ([]uint64, []float32, error) {
	g.mu.RLock()
	defer g.mu.RUnlock()
	if len(vector) == 0 || g.closed.Load() || g.pqPending.Load() {
		return g.cpuIndex.SearchByVectorDistance(vector, dist, maxLimit, allow)
	}
	ap, an, filtered := allowIDs(allow)
	capOut := int64(1 << 12)
	if maxLimit > 0 && maxLimit < capOut {
		capOut = maxLimit
	}
	for {
		ids := make([]uint64, capOut)
		dists := make([]float32, capOut)
		var n C.int64_t
		rc := C.wv_mirror_search_by_distance(g.m, (*C.float)(unsafe.Pointer(&vector[0])), C.int(len(vector)),
			C.float(dist), C.int64_t(maxLimit), filtered, ap, an, (*C.uint64_t)(unsafe.Pointer(&ids[0])),
			(*C.float)(unsafe.Pointer(&dists[0])), C.int64_t(capOut), &n)
		if rc != 0 {
			return g.cpuIndex.SearchByVectorDistance(vector, dist, maxLimit, allow)
		}
		if int64(n) <= capOut {
			return ids[:n], dists[:n], nil
		}
		capOut = int64(n) // the full count is known: one more call with room for it
	}
}

// UpdateUserConfig mirrors hnsw.UpdateUserConfig (config_update.go:79-128): ef,
// dynamic ef and flatSearchCutoff change the search path at once.  Enabling
// PQ starts hnsw's Compress in a goroutine (:97-120 -> compress.go:39-99),
// which ends with the AddPQ record in the commit log and calls the callback:
// from the request on, searches go to the CPU index (it serves uncompressed
// while it fits, then compressed), and each callback flushes the log and
// compacts the mirror -- the compaction that reads the AddPQ record encodes
// every row on the device and serves the codes (wv_mirror.cpp enable_pq),
// with no write needed to trigger it; then the mirror answers again.
func (g *Index) UpdateUserConfig(updated schema.VectorIndexConfig, callback func()) error {
	uc, isUC := updated.(ent.UserConfig)
	g.mu.RLock() // (the mirror is not destroyed under mu)
	enablePQ := isUC && uc.PQ.Enabled && !g.closed.Load() && !g.mirrorCompressed()
	var gen int64
	if enablePQ {
		gen = g.pqGen.Add(1)
		g.pqCalls.Store(0)
		g.pqPending.Store(true)
	}
	g.mu.RUnlock()
	err := g.cpuIndex.UpdateUserConfig(updated, func() {
		callback()
		if enablePQ && g.pqGen.Load() == gen {
			// hnsw calls back once when UpdateUserConfig returns and once when
			// its Compress goroutine ends, with or without an error
			// (config_update.go:113-127): after the second, the log holds the
			// AddPQ record or never will
			final := g.pqCalls.Add(1) >= 2
			go g.syncCompression(gen, final)
		}
	})
	if err != nil {
		if enablePQ {
			g.pqPending.Store(false)
		}
		return err
	}
	g.mu.RLock()
	defer g.mu.RUnlock()
	if isUC && !g.closed.Load() {
		cfg := configOf(uc, g.device)
		C.wv_mirror_update_config(g.m, &cfg)
	}
	return nil
}

// mirrorCompressed: the mirror serves PQ codes (wv_mirror_stats.pq).
func (g *Index) mirrorCompressed() bool {
	var st C.wv_mirror_stats
	return C.wv_mirror_get_stats(g.m, &st) == 0 && st.pq != 0
}

// syncCompression: a flush of the CPU index's log and a compaction, so the
// mirror reads the AddPQ record Compress wrote.  pqPending is cleared once
// the mirror serves the codes, or -- after Compress has ended (final) -- once
// a compaction of the flushed log succeeded without finding one: Compress
// failed, the CPU index stays uncompressed, and so does the mirror.  A
// compaction refused while the mirror is not live (an async startup or a
// resync in flight: WV_ESTALE) is retried, 1 s apart, for up to 10 minutes.
func (g *Index) syncCompression(gen int64, final bool) {
	for try := 0; try < 600; try++ {
		if try > 0 {
			time.Sleep(time.Second)
		}
		if g.pqGen.Load() != gen {
			return // a later enablement owns the flag
		}
		g.mu.Lock()
		if g.closed.Load() {
			g.mu.Unlock()
			return
		}
		err := g.cpuIndex.Flush()
		g.mu.Unlock()
		g.mu.RLock()
		if g.closed.Load() {
			g.mu.RUnlock()
			return
		}
		rc := C.int(C.WV_ESTATE)
		if err == nil {
			rc = C.wv_mirror_compact(g.m)
		}
		compressed := rc == 0 && g.mirrorCompressed()
		g.mu.RUnlock()
		if compressed || (final && rc == 0) {
			if g.pqGen.Load() == gen {
				g.pqPending.Store(false)
			}
			return
		}
		if !final {
			return // (the callback before Compress ends: the final one settles the flag)
		}
	}
}

func (g *Index) close() {
	g.mu.Lock()
	if g.closed.Swap(true) {
		g.mu.Unlock()
		return
	}
	// every call that holds mu shared has returned, and every later one sees
	// closed; mu is released before the destroy, which joins the library's
	// thread (a resync's wvgpuFlush takes mu, then finds closed set)
	g.mu.Unlock()
	if g.metrics != nil {
		g.metrics.stop()
	}
	C.wv_mirror_destroy(g.m) // joins startups / resyncs, waits for a compaction, drains searches
	g.freeHandles()
}

func (g *Index) Shutdown(ctx context.Context) error {
	g.close()
	return g.cpuIndex.Shutdown(ctx)
}

func (g *Index) Drop(ctx context.Context) error {
	g.close()
	return g.cpuIndex.Drop(ctx)
}
