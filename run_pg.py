#!/usr/bin/env python
"""Run a policy-gradient algorithm (`run_pg.py` of the reference) on the MI355X path.

    python run_pg.py --env Hopper-v2 --agent modular_rl_amd.agentzoo.TrpoAgent \
        --n_envs 4096 --horizon 1024 --gamma 0.995 --lam 0.97 --max_kl 0.01 --cg_damping 0.1
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 run_pg.py ...   (data-parallel, RCCL)

Same two-phase argparse as the reference (`run_pg.py:79-102`): GENERAL_OPTIONS +
--env/--agent first, then the agent class's ``options``; ``timestep_limit`` defaults
to the env's max_episode_steps (`run_pg.py:103-105`); ``callback`` prints the
per-iteration stats table (`run_pg.py:126-132`).  ``--use_hdf`` / ``--outfile`` /
``--snapshot_every`` keep the run log and agent snapshots (`run_pg.py:133-142`, as safe
array files, modular_rl_amd/checkpoint.py); ``--load_snapshot`` resumes from one.
"""
import argparse
import json
import os
import sys

import numpy as np
from tabulate import tabulate

from modular_rl_amd.checkpoint import RunLog, load_snapshot, save_snapshot
from modular_rl_amd.core import get_agent_cls, run_policy_gradient_algorithm
from modular_rl_amd.dist import init_from_env
from modular_rl_amd.envs import make
from modular_rl_amd.misc_utils import GENERAL_OPTIONS, update_argument_parser


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    update_argument_parser(parser, GENERAL_OPTIONS)
    parser.add_argument("--env", default="CartPole-v0")
    parser.add_argument("--agent", default="modular_rl_amd.agentzoo.TrpoAgent")
    parser.add_argument("--plot", action="store_true")
    parser.add_argument("--json", action="store_true", help="print stats as JSON lines")
    args, _ = parser.parse_known_args([a for a in argv if a not in ("-h", "--help")])
    env = make(args.env)
    env_spec = env.spec
    agent_ctor = get_agent_cls(args.agent)
    update_argument_parser(parser, agent_ctor.options)
    args = parser.parse_args(argv)
    if args.timestep_limit == 0:
        args.timestep_limit = env_spec.max_episode_steps
    cfg = args.__dict__
    np.random.seed(args.seed)
    comm = init_from_env()
    agent = agent_ctor(env.observation_space, env.action_space, cfg, comm=comm)
    counter = [0]
    if args.load_snapshot:
        meta = load_snapshot(args.load_snapshot, agent)
        counter[0] = int(meta.get("counter", 0))
    log = RunLog(args.outfile, cfg) if (args.use_hdf and comm.rank == 0) else None

    def callback(stats):
        counter[0] += 1
        if comm.rank != 0:
            return
        if log is not None:
            log.record(stats)
            if args.snapshot_every and (counter[0] % args.snapshot_every == 0 or counter[0] == args.n_iter):
                log.snapshot(counter[0], agent, env_spec.id)
                save_snapshot(_snapshot_path(args.outfile, counter[0]), agent, counter[0], env_spec.id)
        if args.json:
            print(json.dumps({k: float(v) for k, v in stats.items() if np.asarray(v).size == 1}), flush=True)
            return
        print("*********** Iteration %i ****************" % counter[0])
        print(tabulate([(k, v) for k, v in stats.items() if np.asarray(v).size == 1]))
        sys.stdout.flush()

    run_policy_gradient_algorithm(env, agent, callback=callback, usercfg=cfg)
    if log is not None:
        log.extra["env_id"] = env_spec.id
        print("Saved results to %s" % log.save())
    env.close()


def _snapshot_path(outfile, counter):
    base = os.path.splitext(outfile)[0]
    return "%s.snap%04i.npz" % (base, counter)


if __name__ == "__main__":
    main()
