"""TEST INFRASTRUCTURE: the CPU oracle (oracle.OracleSystem with set_domain, fp64) running one domain of a decomposed
run, with the same band layout as gcs.domain.EngineDomain ([peer][header + records][4]; the header row's first word
is the band's count) so gcs.domain's transports move either."""
import numpy as np

from gcs.domain import _Domain, in_box

RED = 10  # the engine's allreduce layout (csrc/engine_internal.hpp kDomainRed): reactions [0, 6), shared from RED


class OracleDomain(_Domain):
    def __init__(self, osys, index, boxes, halo, schedule: dict, shared=()):
        super().__init__(index, boxes, halo)
        self.shared = np.asarray(shared, dtype=np.int64).reshape(-1)
        self.o = osys
        self.sched = dict(schedule)
        osys.set_schedule(**dict(schedule, update_wall=0))  # the wall update sees the allreduced reaction
        osys.set_domain(*self.box)
        n = osys.n
        self.cap = n
        npeer = max(1, len(self.peers))
        self.red = np.zeros(RED + 3 * self.shared.size)
        self.glob = np.zeros_like(self.red)
        self.out = np.zeros((npeer, n + 1, 4))
        self.inb = np.zeros_like(self.out)
        self._old = None
        self._flags = 0

    def step(self, st, bd):
        self._old = self.o.get_positions()
        self.o.run(1, first_step=st, temperature=bd["temperature"], timestep=bd["timestep"], seed=bd["seed"])
        c = self.o.get_context()
        self.red[:] = 0.0
        self.red[:3] = c["inward_reaction"]
        self.red[3:6] = c["outward_reaction"]
        if self.shared.size:
            new = self.o.get_positions()[self.shared]
            own = self.owned_mask(self._old[self.shared])
            self.red[RED:] = np.where(own[:, None], new, 0.0).reshape(-1)

    def finish(self):
        # simulation_driver_interphase.cpp:80-90 with the reaction summed over domains
        s = self.sched
        c = self.o.get_context()
        if s.get("update_wall", 0):
            w = np.array(c["wall_semiaxes"])
            R = self.glob[:3] + self.glob[3:6]
            w = w + s["timestep"] * s["wall_mobility"] * (R - np.asarray(s["wall_semiaxes_spring"]) * w)
            c["wall_semiaxes"] = list(w)
        c["inward_reaction"] = list(self.glob[:3])
        c["outward_reaction"] = list(self.glob[3:6])
        self.o.set_context(c)
        if self.shared.size:
            x = self.o.get_positions()
            x[self.shared] = self.glob[RED:].reshape(-1, 3)
            self.o.set_positions(x)

    def pack(self, staged=True):
        new = self.o.get_positions()
        old = self._old
        own = self.owned_mask(old)
        self.out[:, 0, :] = 0.0
        for k, reg in enumerate(self.regions):
            sel = own & (in_box(old, reg) | in_box(new, reg))
            idx = np.nonzero(sel)[0]
            self.out[k, 0, 0] = idx.size
            self.out[k, 1: idx.size + 1, :3] = new[idx]
            self.out[k, 1: idx.size + 1, 3] = idx

    def unpack(self):
        if not self.peers:
            return
        x = self.o.get_positions()
        for k in range(len(self.peers)):
            c = int(self.inb[k, 0, 0])
            idx = self.inb[k, 1: c + 1, 3].astype(np.int64)
            x[idx] = self.inb[k, 1: c + 1, :3]
        self.o.set_positions(x)

    def synchronize(self):
        pass

    def flag_bits(self):
        return self._flags

    def positions(self):
        return self.o.get_positions()

    def context(self):
        return self.o.get_context()
