"""Algorithm ABC and the off-policy trainer loop (mtrl/rl/algorithms/base.py:49-359).

The loop order is the reference's (base.py:157-231): warm-start random actions,
``done = terminations | truncations``, ``final_obs`` substitution, buffer add, then one
update per global step once ``global_step > warmstart_steps``, SPS print every 10 000
steps, evaluation every ``evaluation_frequency`` finished episodes.  When the replay
buffer lives in the same engine as the networks, the sample + update pair runs as ONE
device call (``MTSACEngine.update_many(1)``): no host round trip per gradient step.
At every evaluation the gradient-conflict metrics run on a balanced sample (``compute_weights``,
base.py:279-288): ``config.batch_size`` rows, the reference's 128 per task in every target config.
"""

from __future__ import annotations

import abc
import time
from collections import deque

import numpy as np

from ...types import LogDict


class Algorithm(abc.ABC):
    num_tasks: int

    @staticmethod
    @abc.abstractmethod
    def initialize(config, env_config, seed: int = 1) -> "Algorithm": ...

    @abc.abstractmethod
    def update(self, data) -> tuple["Algorithm", LogDict]: ...

    @abc.abstractmethod
    def get_num_params(self) -> dict[str, int]: ...

    @abc.abstractmethod
    def sample_action(self, observation) -> tuple["Algorithm", np.ndarray]: ...

    @abc.abstractmethod
    def eval_action(self, observations) -> np.ndarray: ...

    def reset(self, env_mask) -> None:  # mtsac.py:286-287
        pass


def _final_obs(infos, done, next_obs):
    if "final_obs" not in infos:
        return next_obs
    fo = infos["final_obs"]
    rows = [fo[i] if (done[i] and fo[i] is not None) else next_obs[i] for i in range(len(done))]
    return np.where(done[:, None], np.stack(rows), next_obs)


class OffPolicyAlgorithm(Algorithm):
    @abc.abstractmethod
    def spawn_replay_buffer(self, env_config, config, seed: int = 1): ...

    def update_from_buffer(self, replay_buffer, batch_size: int, want_logs: bool):
        """sample + update; overridden by engines that sample on the device."""
        return self.update(replay_buffer.sample(batch_size))

    def train(self, config, envs, eval_envs, env_config, run_timestamp: str | None = None, seed: int = 1,
              track: bool = False, checkpoint_manager=None, checkpoint_metadata=None, buffer_checkpoint=None):
        T = self.num_tasks
        global_episodic_return: deque = deque([], maxlen=20 * T)
        global_episodic_length: deque = deque([], maxlen=20 * T)
        obs, _ = envs.reset()
        done = np.full((envs.num_envs,), False)
        start_step, episodes_ended, last_eval_episodes = 0, 0, 0
        if checkpoint_metadata is not None:
            start_step = checkpoint_metadata["step"]
            episodes_ended = checkpoint_metadata["episodes_ended"]
            last_eval_episodes = episodes_ended
        replay_buffer = self.spawn_replay_buffer(env_config, config, seed)
        if buffer_checkpoint is not None:
            replay_buffer.load_checkpoint(buffer_checkpoint)
        self._last_buffer = replay_buffer
        start_time = time.time()
        total_steps = 0
        if track:
            import wandb
        for global_step in range(start_step, config.total_steps // envs.num_envs):
            total_steps = global_step * envs.num_envs
            if global_step < config.warmstart_steps:
                actions = envs.action_space.sample()
            else:
                self, actions = self.sample_action(obs)
            next_obs, rewards, terminations, truncations, infos = envs.step(actions)
            done = np.logical_or(terminations, truncations)
            buffer_obs = _final_obs(infos, done, next_obs)
            replay_buffer.add(obs, buffer_obs, actions, rewards, done)
            obs = next_obs
            for i, env_ended in enumerate(done):
                if env_ended:
                    ep = infos["final_info"]["episode"] if "final_info" in infos else infos["episode"]
                    global_episodic_return.append(ep["r"][i])
                    global_episodic_length.append(ep["l"][i])
                    episodes_ended += 1
            if global_step % 500 == 0 and global_episodic_return:
                mean_ep_return = np.mean(list(global_episodic_return))
                print(f"global_step={total_steps}, mean_episodic_return={mean_ep_return:.4f}")
                if track:
                    wandb.log({"charts/mean_episodic_return": mean_ep_return,
                               "charts/mean_episodic_length": np.mean(list(global_episodic_length))},
                              step=total_steps)
            if global_step > config.warmstart_steps:
                for _ in range(getattr(config, "replay_ratio", 1)):
                    self, logs = self.update_from_buffer(replay_buffer, config.batch_size, want_logs=track)
                    if track:
                        wandb.log(logs, step=total_steps)
                if global_step % 10000 == 0:
                    sps = int((global_step - start_step) * envs.num_envs / (time.time() - start_time))
                    print("SPS:", sps)
                should_eval = (config.evaluation_frequency > 0
                               and episodes_ended - last_eval_episodes >= config.evaluation_frequency
                               and global_step > 0)
                if should_eval:
                    last_eval_episodes = episodes_ended
                    mean_success_rate, mean_returns, per_task = env_config.evaluate(eval_envs or envs, self)
                    eval_metrics = {"charts/mean_success_rate": float(mean_success_rate),
                                    "charts/mean_evaluation_return": float(mean_returns)} | {
                        f"charts/{k}_success_rate": float(v) for k, v in per_task.items()}
                    print(f"total_steps={total_steps}, mean evaluation success rate: {mean_success_rate:.4f}"
                          f" return: {mean_returns:.4f}")
                    if track:
                        wandb.log(eval_metrics, step=total_steps)
                    if hasattr(self, "compute_weights"):  # base.py:279-288
                        # the reference samples envs.num_envs * 128 rows; the engine's batch is
                        # config.batch_size, which is 128 per task in every target config
                        metrics_data = replay_buffer.sample(config.batch_size)
                        self, update_logs = self.compute_weights(metrics_data)
                        if track:
                            wandb.log(update_logs, step=total_steps)
                    if checkpoint_manager is not None:
                        checkpoint_manager.save(total_steps, agent=self, buffer=replay_buffer,
                                                metadata={"timestamp": run_timestamp, "step": global_step,
                                                          "episodes_ended": episodes_ended},
                                                metrics={k.removeprefix("charts/"): v for k, v in eval_metrics.items()})
                    if not eval_envs:
                        obs, _ = envs.reset()
        if global_episodic_return:
            print(f"global_step={total_steps}, mean_episodic_return={np.mean(list(global_episodic_return)):.4f}")
        return self
