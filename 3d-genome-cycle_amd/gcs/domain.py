"""Spatial domain decomposition of ONE trajectory over several devices (C5; DESIGN.md "Multi-GPU").

The reference integrates one system on one thread (md::simulate_brownian_dynamics called from
stage_interphase/simulation_driver_interphase.cpp:57-63); this module splits one such system into boxes, one per
domain (one GPU per rank in production), and keeps the reference's per-step order: force evaluation, Euler-Maruyama
update, then the callback's schedule with the wall update from the step's reaction (:51-52, :80-90), where the
reaction is now the SUM over domains (one allreduce per step).

Geometry: `plan_boxes` bisects the particles recursively (k-d style: each cut along the longest extent of the
particles it splits, at the count quantile), so 8 domains are 2 x 2 x 2 blocks of equal bead counts whose sides stay
several halos thick; `plan_slabs` cuts z only.  The boxes tile space (outer faces at +-inf).

Protocol (kernels in csrc/domain.hip, which proves the invariants):
  * every domain holds all N particles by global index; domain d OWNS the particles inside its box [lo_d, hi_d) at
    the start of a step and integrates only those (Philox noise is keyed by the global index, so a particle draws
    the same noise whichever domain owns it);
  * domain d bins only the particles inside its region E_d = [lo_d - halo, hi_d + halo); `halo` exceeds the list
    radius (pair cutoff + skin), the droplet cutoff and the longest bond (the pack kernel checks the bonds every
    step, the list step's tail the displacement since the last build);
  * after every step d sends each peer p the owned particles whose old or new position lies in E_p; p writes them
    into both of its position buffers (and its list slots).  Peers are the domains whose regions overlap.

Every exchange buffer is the engine's own (gcs_engine_domain_buffers): a band per peer whose first row holds its
count, so one message per peer carries both, and the reaction/shared-position buffer of the allreduce.

Transports:
  * `RcclRun` -- production, one domain per GPU: the engine itself issues ncclAllReduce and one grouped
    ncclSend/ncclRecv per peer on its HIP stream (gcs_engine_domain_run), chunks of steps captured in a hipGraph; the
    host only hands the communicator id to the ranks (torch.distributed object broadcast, CPU).
  * `LocalTransport` -- several domains in one process on one device: the reaction summed on the host in domain
    order, the bands copied device-to-device between the engines (gcs_engine_domain_receive).
  * `DistTransport` -- host-staged over torch.distributed (gloo, CPU tensors): any process layout, including several
    processes sharing one device (RCCL refuses two ranks on one GPU); also the transport of the CPU oracle domains
    the tests use (tests/oracle_domain.py).
"""
from __future__ import annotations

import numpy as np

from .config import InterphaseConfig

FLAG_BOND = 1       # a bond of an owned particle is longer than the halo (its partner may be stale)
FLAG_CAPACITY = 2   # a band exceeded the exchange buffer capacity
FLAG_LOST = 4       # a particle owned by no domain's lists (it moved further than the halo between list builds)
FLAG_MOTION = 8     # pair cutoff + largest displacement since the last list build exceeds the halo


class DomainError(RuntimeError):
    pass


def _f32(v):
    """a cut the device compares exactly (its boxes are fp32)"""
    return float(np.float32(v))


def _open_box():
    return (np.full(3, -np.inf), np.full(3, np.inf))


def plan_slabs(z, ndom: int):
    """Equal-count z-slabs of the current positions as boxes [(lo[3], hi[3])], x and y open, outer z ends open."""
    z = np.asarray(z, dtype=np.float64)
    if ndom < 1:
        raise ValueError("need at least one domain")
    cuts = np.quantile(z, np.arange(1, ndom) / ndom) if ndom > 1 else np.array([])
    edges = np.concatenate([[-np.inf], [_f32(c) for c in cuts], [np.inf]])
    out = []
    for d in range(ndom):
        lo, hi = _open_box()
        lo[2], hi[2] = edges[d], edges[d + 1]
        out.append((lo, hi))
    return out


def plan_boxes(x, ndom: int):
    """Recursive bisection of the current positions into `ndom` boxes of equal particle counts (+-1): each cut runs
    across the longest extent of the particles it splits, at the count quantile k1 / k (k1 = k // 2 of the k domains
    go below it).  8 domains of a compact nucleus are 2 x 2 x 2 blocks.  Boxes [(lo[3], hi[3])], outer faces open."""
    x = np.asarray(x, dtype=np.float64)[:, :3]
    if ndom < 1:
        raise ValueError("need at least one domain")
    out = []

    def split(idx, lo, hi, k):
        if k == 1:
            out.append((lo.copy(), hi.copy()))
            return
        if idx.size < k:
            raise ValueError("fewer particles than domains")
        pts = x[idx]
        ax = int(np.argmax(pts.max(axis=0) - pts.min(axis=0)))
        k1 = k // 2
        v = np.sort(pts[:, ax])
        m = min(max(int(round(v.size * k1 / k)), 1), v.size - 1)
        cut = _f32(0.5 * (v[m - 1] + v[m]))
        below = x[idx, ax] < cut
        hi1 = hi.copy()
        hi1[ax] = cut
        lo2 = lo.copy()
        lo2[ax] = cut
        split(idx[below], lo, hi1, k1)
        split(idx[~below], lo2, hi, k - k1)

    split(np.arange(x.shape[0]), *_open_box(), ndom)
    return out


BOND_SIGMAS = 7.5  # a chain bond stretched beyond this many thermal widths: ~1e-11 per bond-step


LIST_SKIN = 0.5  # the list step's largest default skin / pair cutoff (GCS_OPT_LIST_SKIN: 500 per mille fp32, 350 fp64)


def domain_halo(cfg: InterphaseConfig, margin: float = 0.05, list_skin: float = LIST_SKIN) -> float:
    """The reach a domain must see fresh beyond its box: the list radius, pair cutoff at core_scale 1
    (simulation_driver_forcefield.cpp:25-28) + the list skin (list_skin x cutoff; 0: the tile step's halo), and the
    chain bonds' reach l + 7.5 sqrt(T / K) at bond_scale 1 (:71-83; semispring, INFERRED form), plus a margin for one
    step's displacement.  The nucleolar bonds and the droplet act among SHARED particles only (shared_particles),
    which every domain holds fresh."""
    rc = max(cfg.a_core_diameter, cfg.b_core_diameter)
    reach = rc * (1.0 + list_skin)
    for k, l in ((cfg.a_core_bond_spring, cfg.a_core_bond_length), (cfg.b_core_bond_spring, cfg.b_core_bond_length)):
        if k > 0:
            reach = max(reach, l + BOND_SIGMAS * float(np.sqrt(cfg.temperature / k)))
    return reach + margin


def shared_particles(design):
    """The nucleolar beads and their NOR beads (simulation_driver_forcefield.cpp:140-186): their bonds
    (nucleolus_bond_spring 10) and the droplet (cutoff 0.4) reach beyond any practical halo."""
    b = np.asarray(design.nucleolar_bonds, dtype=np.int64).reshape(-1, 2)
    return np.unique(b.reshape(-1))


def region(box, halo):
    """a box extended by the halo on every face"""
    return (np.asarray(box[0], dtype=np.float64) - halo, np.asarray(box[1], dtype=np.float64) + halo)


def in_box(x, box):
    """mask of the rows of x inside box [lo, hi) (per axis)"""
    x = np.asarray(x)[:, :3]
    return np.all((x >= np.asarray(box[0])) & (x < np.asarray(box[1])), axis=1)


def peers_of(d: int, boxes, halo: float):
    """Domains whose regions overlap d's (symmetric; touching counts, so the engines' fp32 regions can never overlap
    where these do not)."""
    lo, hi = region(boxes[d], halo)
    out = []
    for p, b in enumerate(boxes):
        if p == d:
            continue
        plo, phi = region(b, halo)
        if np.all(plo <= hi + 1e-5) and np.all(lo <= phi + 1e-5):
            out.append(p)
    return out


def band_capacity(x, boxes, halo, d, margin: float = 1.5, floor: int = 1024) -> int:
    """Records per band for domain d: its particles inside the largest peer region at the start, times `margin`
    (the bands drift slowly; an overflow is flagged on the device and raised by check()), at least `floor`."""
    x = np.asarray(x)
    mine = in_box(x, boxes[d])
    most = 0
    for p in peers_of(d, boxes, halo):
        most = max(most, int((mine & in_box(x, region(boxes[p], halo))).sum()))
    return int(min(x.shape[0], max(floor, np.ceil(margin * most))))


def _finite(v):
    return np.clip(np.asarray(v, dtype=np.float64), -3.0e38, 3.0e38)


class _Domain:
    def __init__(self, index, boxes, halo):
        self.index = index
        self.ndom = len(boxes)
        self.box = (np.asarray(boxes[index][0], dtype=np.float64), np.asarray(boxes[index][1], dtype=np.float64))
        self.halo = halo
        self.peers = peers_of(index, boxes, halo)
        self.peer_boxes = [boxes[p] for p in self.peers]
        self.regions = [tuple(_finite(v) for v in region(boxes[p], halo)) for p in self.peers]

    def owned_mask(self, x):
        return in_box(x, self.box)


class EngineDomain(_Domain):
    """A gcs.engine.Engine running one domain with its own exchange buffers (no torch tensors: host staging in numpy
    for the host-staged transports, device-to-device or RCCL otherwise)."""

    def __init__(self, engine, index, boxes, halo, cap=None, shared=()):
        super().__init__(index, boxes, halo)
        self.shared = np.asarray(shared, dtype=np.int64).reshape(-1)
        self.e = engine
        n = engine.n
        self.cap = int(cap if cap is not None else n)
        engine.set_domain(self.box, halo, self.peer_boxes, index, self.ndom)
        engine.set_domain_shared(self.shared)
        self.nred = engine.domain_buffers(self.cap)
        npeer = max(1, len(self.peers))
        # local reduction (10) + shared particles' positions + one displacement slot per domain (csrc/domain.hip)
        self.red = np.zeros(self.nred)
        self.glob = np.zeros(self.nred)  # its sum over domains
        # host staging: [peer][header + cap][4] records in the engine's precision (csrc/domain.hip)
        self.out = np.zeros((npeer, self.cap + 1, 4), dtype=np.float64 if engine.precision == 64 else np.float32)
        self.inb = np.zeros_like(self.out)

    def step(self, st, bd):
        self.e.domain_step_host(st, self.red, **bd)

    def finish(self):
        self.e.domain_finish_host(self.glob)

    def pack(self, staged=True):
        self.e.domain_pack_host(self.out if staged else None)

    def unpack(self):
        self.e.domain_unpack_host(self.inb)

    def band_count(self, k):
        return int(self.out[k, 0, :1].view(np.int32)[0])

    def synchronize(self):
        self.e.synchronize()

    def flag_bits(self):
        return self.e.domain_flags()

    def positions(self):
        return self.e.get_positions()

    def context(self):
        return self.e.get_context()


class LocalTransport:
    """All domains in this process (indexed by domain number): the reaction summed in domain order on the host;
    engine bands move device-to-device (one device), other domains' through their host arrays."""

    def __init__(self, domains):
        self.domains = domains
        self.device = all(isinstance(d, EngineDomain) for d in domains)

    def allreduce(self):
        tot = self.domains[0].red.copy()
        for d in self.domains[1:]:
            tot += d.red
        for d in self.domains:
            d.glob[:] = tot

    def pack(self):
        for d in self.domains:
            d.pack(staged=False) if self.device else d.pack()

    def exchange(self):
        for d in self.domains:
            for k, p in enumerate(d.peers):
                q = self.domains[p]
                kk = q.peers.index(d.index)
                if self.device:
                    q.e.domain_receive(kk, d.e, k)
                else:
                    q.inb[kk] = d.out[k]

    def unpack(self):
        for d in self.domains:
            d.e.domain_unpack_received() if self.device else d.unpack()


class DistTransport:
    """One domain per rank over torch.distributed with host staging (gloo, CPU tensors): the reaction allreduce and
    one send/recv of the band with each peer."""

    def __init__(self, domain, dist):
        self.d = domain
        self.dist = dist

    def allreduce(self):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(self.d.red, dtype=np.float64))
        self.dist.all_reduce(t)
        self.d.glob[:] = t.numpy()

    def pack(self):
        self.d.pack()

    def exchange(self):
        import torch
        d, dist = self.d, self.dist
        if not d.peers:
            return
        ops, recv = [], []
        for k, p in enumerate(d.peers):
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(d.out[k])), p))
            r = torch.empty(d.inb[k].shape, dtype=torch.from_numpy(d.inb[k]).dtype)
            recv.append(r)
            ops.append(dist.P2POp(dist.irecv, r, p))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for k, r in enumerate(recv):
            d.inb[k] = r.numpy()

    def unpack(self):
        self.d.unpack()


class RcclRun:
    """Production decomposed run: one EngineDomain per rank (one GPU each), the whole step sequence -- kernels,
    ncclAllReduce of the reaction, grouped ncclSend/ncclRecv of the bands -- issued by the engine on its stream
    (gcs_engine_domain_run); torch.distributed (any backend) only carries the communicator id at setup."""

    def __init__(self, domain: EngineDomain, dist=None):
        """dist: torch.distributed (any backend) to hand the communicator id to the ranks; None: one rank."""
        from .engine import rccl_unique_id
        self.d = domain
        self.domains = [domain]
        rank, world = (dist.get_rank(), dist.get_world_size()) if dist is not None else (0, 1)
        box = [rccl_unique_id() if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(box, src=0)
        domain.e.domain_rccl(box[0], world, rank, domain.peers)

    def run(self, steps, first_step=0, temperature=1.0, timestep=1e-5, seed=0):
        self.d.e.domain_run(steps, first_step=first_step, temperature=temperature, timestep=timestep, seed=seed)

    def check(self):
        _raise_flags(self.d.flag_bits())

    def local_positions(self, n):
        return DecomposedRun.local_positions(self, n)


def _raise_flags(bits):
    if bits & FLAG_BOND:
        raise DomainError("a bond is longer than the domain halo: raise the halo")
    if bits & FLAG_CAPACITY:
        raise DomainError("a band exceeded the exchange buffer capacity: raise cap")
    if bits & (FLAG_LOST | FLAG_MOTION):
        raise DomainError("particles moved further than the halo allows between list builds: raise the halo")


class DecomposedRun:
    """Steps of one trajectory split over domains, driven from the host: step -> allreduce(reaction) -> finish ->
    pack -> exchange -> unpack.  `domains`: the domains of this process; `transport`: LocalTransport or
    DistTransport (RcclRun drives the same sequence from inside the engine)."""

    def __init__(self, domains, transport):
        self.domains = list(domains)
        self.tr = transport

    def run(self, steps, first_step=0, temperature=1.0, timestep=1e-5, seed=0):
        bd = {"temperature": temperature, "timestep": timestep, "seed": seed}
        for st in range(first_step, first_step + steps):
            for d in self.domains:
                d.step(st, bd)
            self.tr.allreduce()
            for d in self.domains:
                d.finish()
            self.tr.pack()
            self.tr.exchange()
            self.tr.unpack()

    def check(self):
        bits = 0
        for d in self.domains:
            bits |= d.flag_bits()
        _raise_flags(bits)

    def local_positions(self, n):
        """(positions, owned mask) of this process's domains, each particle taken from its owner."""
        x = np.zeros((n, 3))
        m = np.zeros(n, dtype=bool)
        for d in self.domains:
            xd = d.positions()
            own = d.owned_mask(xd)
            x[own] = xd[own]
            m |= own
        return x, m


def gather_positions(run, n: int, dist=None):
    """Whole-system positions from the owners (every particle owned exactly once)."""
    x, m = run.local_positions(n)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        import torch
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, (x, m))
        cnt = np.zeros(n, dtype=np.int64)
        x = np.zeros((n, 3))
        for xp, mp in parts:
            x[mp] = xp[mp]
            cnt += mp
        if not (cnt == 1).all():
            raise DomainError("ownership is not a partition")
        return x
    if not m.all():
        raise DomainError("ownership is not a partition")
    return x
