"""Spatial domain decomposition of ONE trajectory over several devices (C5; DESIGN.md "Multi-GPU").

The reference integrates one system on one thread (md::simulate_brownian_dynamics called from
stage_interphase/simulation_driver_interphase.cpp:57-63); this module splits one such system into z-slabs, one per
domain (one GPU per rank in production), and keeps the reference's per-step order: force evaluation, Euler-Maruyama
update, then the callback's schedule with the wall update from the step's reaction (:51-52, :80-90), where the
reaction is now the SUM over domains (one allreduce of 6 doubles per step).

Protocol (kernels in csrc/domain.hip, which proves the invariants):
  * every domain holds all N particles by global index; domain d OWNS the particles whose z lies in its slab
    [lo_d, hi_d) at the start of a step and integrates only those (Philox noise is keyed by the global index, so a
    particle draws the same noise whichever domain owns it);
  * domain d bins only the particles inside its region E_d = [lo_d - halo, hi_d + halo); `halo` exceeds the pair
    cutoff, the droplet cutoff and the longest bond (the pack kernel checks the bonds every step);
  * after every step d sends each peer p the owned particles whose old or new z lies in E_p; p writes them into
    both of its position buffers.  Peers are the domains whose regions overlap (possibly more than the two
    neighbours when slabs are thinner than the halo).

Backends: `EngineDomain` (the HIP engine; buffers are torch device tensors whose pointers go through the C ABI;
torch's device runtime must be initialised before libgcs.so is loaded, so both share one HIP runtime)
and `OracleDomain` (tests only: the CPU oracle, one step per call).  Transports: `LocalTransport` (all domains in
one process, e.g. several engines on one GPU for parity tests) and `DistTransport` (one domain per rank over
torch.distributed: RCCL for engines, ordered on the engine's HIP stream; gloo for the CPU oracle tests).
"""
from __future__ import annotations

import numpy as np

from .config import InterphaseConfig

FLAG_BOND = 1       # a bond of an owned particle is longer than the halo (its partner may be stale)
FLAG_CAPACITY = 2   # a band exceeded the exchange buffer capacity


class DomainError(RuntimeError):
    pass


def plan_slabs(z, ndom: int):
    """Equal-count z-slabs of the current positions: [(lo, hi)] with open outer ends."""
    z = np.asarray(z, dtype=np.float64)
    if ndom < 1:
        raise ValueError("need at least one domain")
    cuts = np.quantile(z, np.arange(1, ndom) / ndom) if ndom > 1 else np.array([])
    edges = np.concatenate([[-np.inf], cuts, [np.inf]])
    return [(float(edges[d]), float(edges[d + 1])) for d in range(ndom)]


BOND_SIGMAS = 7.5  # a chain bond stretched beyond this many thermal widths: ~1e-11 per bond-step


def domain_halo(cfg: InterphaseConfig, margin: float = 0.05) -> float:
    """The reach a domain must see fresh beyond its slab: the pair cutoff at core_scale 1
    (simulation_driver_forcefield.cpp:25-28) and the chain bonds' reach l + 7.5 sqrt(T / K) at bond_scale 1
    (:71-83; semispring, INFERRED form), plus a margin for one step's displacement.  The nucleolar bonds and the
    droplet act among SHARED particles only (shared_particles), which every domain holds fresh."""
    rc = max(cfg.a_core_diameter, cfg.b_core_diameter)
    for k, l in ((cfg.a_core_bond_spring, cfg.a_core_bond_length), (cfg.b_core_bond_spring, cfg.b_core_bond_length)):
        if k > 0:
            rc = max(rc, l + BOND_SIGMAS * float(np.sqrt(cfg.temperature / k)))
    return rc + margin


def shared_particles(design):
    """The nucleolar beads and their NOR beads (simulation_driver_forcefield.cpp:140-186): their bonds
    (nucleolus_bond_spring 10) and the droplet (cutoff 0.4) reach beyond any practical halo."""
    b = np.asarray(design.nucleolar_bonds, dtype=np.int64).reshape(-1, 2)
    return np.unique(b.reshape(-1))


def region(slab, halo):
    return (slab[0] - halo, slab[1] + halo)


def peers_of(d: int, slabs, halo: float):
    """Domains whose regions overlap d's (symmetric)."""
    lo, hi = region(slabs[d], halo)
    out = []
    for p, s in enumerate(slabs):
        if p == d:
            continue
        plo, phi = region(s, halo)
        if plo < hi and lo < phi:
            out.append(p)
    return out


def _finite(v):
    return float(np.clip(v, -3.0e38, 3.0e38))


class _Domain:
    def __init__(self, index, slabs, halo):
        self.index = index
        self.slab = slabs[index]
        self.halo = halo
        self.peers = peers_of(index, slabs, halo)
        self.regions = [tuple(_finite(v) for v in region(slabs[p], halo)) for p in self.peers]

    def owned_mask(self, x):
        z = np.asarray(x)[:, 2]
        return (z >= self.slab[0]) & (z < self.slab[1])


class EngineDomain(_Domain):
    """A gcs.engine.Engine running one domain; exchange buffers are torch tensors on the engine's device."""

    def __init__(self, engine, index, slabs, halo, cap=None, device=None, shared=()):
        import torch
        super().__init__(index, slabs, halo)
        self.shared = np.asarray(shared, dtype=np.int64).reshape(-1)
        self.e = engine
        self.torch = torch
        self.device = torch.device("cuda", device if device is not None else torch.cuda.current_device())
        n = engine.n
        self.cap = int(cap if cap is not None else n)
        npeer = max(1, len(self.peers))
        f64, f32, i32 = torch.float64, torch.float32, torch.int32
        nred = 8 + 3 * self.shared.size  # local reduction + shared particles' positions (csrc/domain.hip)
        self.red = torch.zeros(nred, dtype=f64, device=self.device)
        self.glob = torch.zeros(nred, dtype=f64, device=self.device)
        self.out = torch.zeros((npeer, self.cap, 4), dtype=f32, device=self.device)
        self.counts = torch.zeros(npeer, dtype=i32, device=self.device)
        self.inb = torch.zeros_like(self.out)
        self.inc = torch.zeros_like(self.counts)
        self.flags = torch.zeros(1, dtype=i32, device=self.device)
        lo, hi = (_finite(v) for v in self.slab)
        engine.set_domain(lo, hi, halo, self.regions)
        engine.set_domain_shared(self.shared)
        self._stream = None

    def stream(self):
        """The engine's HIP stream as a torch stream (collectives are ordered on it, no host synchronisation)."""
        if self._stream is None:
            self._stream = self.torch.cuda.ExternalStream(self.e.stream_handle(), device=self.device)
        return self._stream

    def step(self, st, bd):
        self.e.domain_step(st, self.red.data_ptr(), **bd)

    def finish(self):
        self.e.domain_finish(self.glob.data_ptr())

    def pack(self):
        self.e.domain_pack(self.out.data_ptr(), self.counts.data_ptr(), self.cap, self.flags.data_ptr())

    def unpack(self):
        self.e.domain_unpack(self.inb.data_ptr(), self.inc.data_ptr(), len(self.peers), self.cap)

    def synchronize(self):
        self.e.synchronize()

    def flag_bits(self):
        self.e.synchronize()
        return int(self.flags.item())

    def positions(self):
        return self.e.get_positions()

    def context(self):
        return self.e.get_context()


class OracleDomain(_Domain):
    """TEST INFRASTRUCTURE: the CPU oracle running one domain (oracle.OracleSystem with set_domain), fp64."""

    def __init__(self, osys, index, slabs, halo, schedule: dict, shared=()):
        import torch
        super().__init__(index, slabs, halo)
        self.shared = np.asarray(shared, dtype=np.int64).reshape(-1)
        self.o = osys
        self.torch = torch
        self.sched = dict(schedule)
        osys.set_schedule(**dict(schedule, update_wall=0))  # the wall update sees the allreduced reaction
        lo, hi = self.slab
        osys.set_domain(lo, hi)
        n = osys.n
        self.cap = n
        npeer = max(1, len(self.peers))
        self.red = torch.zeros(8 + 3 * self.shared.size, dtype=torch.float64)
        self.glob = torch.zeros_like(self.red)
        self.out = torch.zeros((npeer, n, 4), dtype=torch.float64)
        self.counts = torch.zeros(npeer, dtype=torch.int32)
        self.inb = torch.zeros_like(self.out)
        self.inc = torch.zeros_like(self.counts)
        self._old = None
        self._flags = 0

    def step(self, st, bd):
        self._old = self.o.get_positions()
        self.o.run(1, first_step=st, temperature=bd["temperature"], timestep=bd["timestep"], seed=bd["seed"])
        c = self.o.get_context()
        self.red[:3] = self.torch.tensor(c["inward_reaction"], dtype=self.torch.float64)
        self.red[3:6] = self.torch.tensor(c["outward_reaction"], dtype=self.torch.float64)
        if self.shared.size:
            new = self.o.get_positions()[self.shared]
            own = self.owned_mask(self._old[self.shared])
            self.red[8:] = self.torch.from_numpy(np.where(own[:, None], new, 0.0).reshape(-1))

    def finish(self):
        # simulation_driver_interphase.cpp:80-90 with the reaction summed over domains
        s = self.sched
        c = self.o.get_context()
        if s.get("update_wall", 0):
            w = np.array(c["wall_semiaxes"])
            R = self.glob[:3].numpy() + self.glob[3:6].numpy()
            w = w + s["timestep"] * s["wall_mobility"] * (R - np.asarray(s["wall_semiaxes_spring"]) * w)
            c["wall_semiaxes"] = list(w)
        c["inward_reaction"] = list(self.glob[:3].numpy())
        c["outward_reaction"] = list(self.glob[3:6].numpy())
        self.o.set_context(c)
        if self.shared.size:
            x = self.o.get_positions()
            x[self.shared] = self.glob[8:].numpy().reshape(-1, 3)
            self.o.set_positions(x)

    def pack(self):
        new = self.o.get_positions()
        old = self._old
        own = self.owned_mask(old)
        self.counts.zero_()
        for k, (lo, hi) in enumerate(self.regions):
            sel = own & (((old[:, 2] >= lo) & (old[:, 2] < hi)) | ((new[:, 2] >= lo) & (new[:, 2] < hi)))
            idx = np.nonzero(sel)[0]
            self.out[k, : idx.size, :3] = self.torch.from_numpy(new[idx])
            self.out[k, : idx.size, 3] = self.torch.from_numpy(idx.astype(np.float64))
            self.counts[k] = int(idx.size)

    def unpack(self):
        if not self.peers:
            return
        x = self.o.get_positions()
        for k in range(len(self.peers)):
            c = int(self.inc[k])
            idx = self.inb[k, :c, 3].numpy().astype(np.int64)
            x[idx] = self.inb[k, :c, :3].numpy()
        self.o.set_positions(x)

    def synchronize(self):
        pass

    def flag_bits(self):
        return self._flags

    def positions(self):
        return self.o.get_positions()

    def context(self):
        return self.o.get_context()


class LocalTransport:
    """All domains in this process (indexed by domain number).  Fixed-order reaction sum; host-synchronous."""

    def __init__(self, domains):
        self.domains = domains

    def _sync(self):
        for d in self.domains:
            d.synchronize()
        t = self.domains[0].torch
        if t.cuda.is_available():
            t.cuda.synchronize()

    def allreduce(self):
        self._sync()
        tot = self.domains[0].red.clone()
        for d in self.domains[1:]:
            tot += d.red.to(tot.device)
        for d in self.domains:
            d.glob.copy_(tot)
        self._sync()

    def exchange(self):
        self._sync()
        for d in self.domains:
            for k, p in enumerate(d.peers):
                q = self.domains[p]
                kk = q.peers.index(d.index)
                q.inb[kk].copy_(d.out[k])
                q.inc[kk] = d.counts[k]
        self._sync()


class DistTransport:
    """One domain per rank over torch.distributed: RCCL (backend "nccl") for engines, with the collectives
    ordered on the engine's HIP stream (no host synchronisation); gloo for CPU (oracle) domains."""

    def __init__(self, domain, dist):
        self.d = domain
        self.dist = dist
        self.gpu = isinstance(domain, EngineDomain)
        if self.gpu and dist.get_backend() != "nccl":
            raise DomainError("engine domains exchange over RCCL (backend 'nccl')")

    def _on_stream(self):
        import contextlib
        return self.d.torch.cuda.stream(self.d.stream()) if self.gpu else contextlib.nullcontext()

    def allreduce(self):
        with self._on_stream():
            self.d.glob.copy_(self.d.red)
            self.dist.all_reduce(self.d.glob)

    def exchange(self):
        d, dist = self.d, self.dist
        if not d.peers:
            return
        with self._on_stream():
            ops = []
            for k, p in enumerate(d.peers):
                ops.append(dist.P2POp(dist.isend, d.out[k], p))
                ops.append(dist.P2POp(dist.isend, d.counts[k:k + 1], p))
                ops.append(dist.P2POp(dist.irecv, d.inb[k], p))
                ops.append(dist.P2POp(dist.irecv, d.inc[k:k + 1], p))
            for r in dist.batch_isend_irecv(ops):
                r.wait()


class DecomposedRun:
    """Steps of one trajectory split over domains: step -> allreduce(reaction) -> finish -> pack -> exchange ->
    unpack.  `domains`: the domains of this process; `transport`: LocalTransport or DistTransport."""

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
            for d in self.domains:
                d.pack()
            self.tr.exchange()
            for d in self.domains:
                d.unpack()

    def check(self):
        bits = 0
        for d in self.domains:
            bits |= d.flag_bits()
        if bits & FLAG_BOND:
            raise DomainError("a bond is longer than the domain halo: raise the halo")
        if bits & FLAG_CAPACITY:
            raise DomainError("a band exceeded the exchange buffer capacity: raise cap")

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


def gather_positions(run: DecomposedRun, n: int, dist=None):
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
