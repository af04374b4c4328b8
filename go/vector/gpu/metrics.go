//go:build linux && cgo

package gpu

// Gauges of the GPU mirror, in the pattern of hnsw's per-index metrics
// (adapters/repos/db/vector/hnsw/metrics.go:23-228: class_name / shard_name
// labels on vectors registered once per process).  A goroutine samples
// wv_mirror_get_stats every few seconds; nothing is added to the search path.

/*
#include "wvgpu.h"
*/
import "C"

import (
	"sync"
	"time"

	"github.com/prometheus/client_golang/prometheus"
)

var (
	metricsOnce sync.Once
	gpuGauges   *prometheus.GaugeVec
)

func registerGauges() {
	gpuGauges = prometheus.NewGaugeVec(prometheus.GaugeOpts{
		Name: "vector_index_gpu_mirror",
		Help: "GPU mirror of a shard's hnsw index: state (0 idle, 1 starting, 2 live, 3 stale), rows, " +
			"delta rows, graph nodes, capacity, compactions, resyncs, mean micro-batch, PQ",
	}, []string{"class_name", "shard_name", "quantity"})
	if err := prometheus.Register(gpuGauges); err != nil {
		if are, ok := err.(prometheus.AlreadyRegisteredError); ok {
			gpuGauges = are.ExistingCollector.(*prometheus.GaugeVec)
		}
	}
}

type mirrorMetrics struct {
	done chan struct{}
	wg   sync.WaitGroup
}

func newMirrorMetrics(g *Index, className, shardName string) *mirrorMetrics {
	metricsOnce.Do(registerGauges)
	mm := &mirrorMetrics{done: make(chan struct{})}
	set := func(q string, v float64) {
		gpuGauges.With(prometheus.Labels{"class_name": className, "shard_name": shardName, "quantity": q}).Set(v)
	}
	mm.wg.Add(1)
	go func() {
		defer mm.wg.Done()
		t := time.NewTicker(5 * time.Second)
		defer t.Stop()
		for {
			select {
			case <-mm.done:
				return
			case <-t.C:
			}
			var st C.wv_mirror_stats
			g.mu.RLock()
			if g.closed.Load() {
				g.mu.RUnlock()
				return
			}
			rc := C.wv_mirror_get_stats(g.m, &st)
			g.mu.RUnlock()
			if rc != 0 {
				continue
			}
			set("state", float64(st.state))
			set("rows", float64(st.n_rows))
			set("delta_rows", float64(st.delta_rows))
			set("graph_nodes", float64(st.graph_nodes))
			set("capacity", float64(st.capacity))
			set("compactions", float64(st.compactions))
			set("resyncs", float64(st.resyncs))
			set("pq", float64(st.pq))
			if st.batcher_batches > 0 {
				set("mean_batch", float64(st.batcher_requests)/float64(st.batcher_batches))
			}
		}
	}()
	return mm
}

func (mm *mirrorMetrics) stop() {
	close(mm.done)
	mm.wg.Wait()
}
