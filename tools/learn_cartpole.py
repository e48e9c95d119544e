"""Run the reference's learn() loop (trpo_inksci.py:89-177) on CartPole-v0 on the GPU and print the
reference's per-iteration statistics.  usage: python tools/learn_cartpole.py [iterations] [n_envs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from trpo_amd import TRPOAgent  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 60
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
agent = TRPOAgent(4, 2, hidden=(64,), max_rows=8192)
t0 = time.time()
hist = agent.learn(max_iterations=iters, n_envs=n_envs, seed=1)
dt = time.time() - t0
print(f"\n{len(hist)} iterations in {dt:.2f} s ({1000 * dt / max(1, len(hist)):.1f} ms/iteration, n_envs={n_envs})")
print("mean episode reward per iteration:", " ".join(f"{h['reward_mean']:.0f}" for h in hist))
