"""Host mirror of formation 0 for playback.

visualize_policy.py:37-46 animates ``env.formationsim_list[0].fig`` while stepping the env.
The figure drawn here shows the same scene as the reference's FormationSimulator window
(simulate.py:33-59, 63-67): the 400x600 box, one dot per agent, a thin segment from each agent
to its ring successor, and the goal.  It is refreshed from a D2H copy of formation 0 only.
"""
from __future__ import annotations

import numpy as np


class FormationFigure:
    def __init__(self, num_agents: int, width: float = 400, height: float = 600):
        import matplotlib.pyplot as plt

        self.num_agents = int(num_agents)
        self.fig = plt.figure(figsize=(width / 100, height / 100))
        self.ax = self.fig.add_subplot(111)
        m = 10
        self.ax.set_xlim(-m, width + m)
        self.ax.set_ylim(-m, height + m)
        self.ax.plot([0, width, width, 0, 0], [0, 0, height, height, 0], color="black")
        self.dots = []
        self.links = []
        for _ in range(self.num_agents):
            c = plt.Circle((0, 0), radius=2, color="blue")
            self.ax.add_artist(c)
            self.dots.append(c)
            ln = plt.Line2D([0, 0], [0, 0], color="blue", linewidth=0.2)
            self.ax.add_artist(ln)
            self.links.append(ln)
        self.goal = plt.Circle((0, 0), radius=10, color="red")
        self.ax.add_artist(self.goal)

    def update(self, px: np.ndarray, py: np.ndarray, gx: float, gy: float) -> None:
        nx_ = np.roll(px, -1)
        ny_ = np.roll(py, -1)
        for k in range(self.num_agents):
            self.dots[k].center = (float(px[k]), float(py[k]))
            self.links[k].set_data([float(px[k]), float(nx_[k])], [float(py[k]), float(ny_[k])])
        self.goal.center = (float(gx), float(gy))
