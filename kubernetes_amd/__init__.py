"""kubernetes_amd — MI355X-native kube-scheduler Filter/Score pass.

The hot path of smarterclayton/kubernetes v0.13.0-dev's generic scheduler
(pkg/scheduler: findNodesThatFit / prioritizeNodes / selectHost) rebuilt as
CDNA4 HIP kernels behind a C ABI (include/kschedgpu.h, libkschedgpu.so), with a
host-side mirror of the reference's algorithm API:

  factory      predicate/priority registry, DefaultProvider, Policy -> ksg_config
  scheduler    GPUScheduler (algorithm.Scheduler drop-in), FitError, listers
  modeler      cache.Store, SimpleModeler (AssumePod = the commit), PodMirror (event-driven device state)
  ingest       api objects -> interned SoA arrays
  engine       one libkschedgpu.so context (DeviceScheduler)
  api/resource/labels   the pkg/api, resource.Quantity and labels subset the path reads
  workload     seeded synthetic scheduler_perf-style clusters (BASELINE configs)
"""
__version__ = "0.1.0"
