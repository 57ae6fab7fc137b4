"""Re-render the sender-pane crops kat_gif_ports.json was transcribed from.

Runs only in the build container (it reads /root/reference/images, which never
travels to the GPU box); writes PNG strips for a human to re-read the ports:

    python tests/golden/gif_ports_crops.py /tmp/gif_ports
"""
import os
import sys

from PIL import Image

REF = "/root/reference/images"


def strip(gif, frames, box, out):
    im = Image.open(os.path.join(REF, gif))
    crops = []
    for i in frames:
        im.seek(i)
        crops.append(im.convert("RGB").crop(box))
    w, h = crops[0].size
    s = Image.new("RGB", (w * len(crops), h))
    for j, c in enumerate(crops):
        s.paste(c, (w * j, 0))
    s.save(out)


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    im = Image.open(os.path.join(REF, "test1.gif"))
    last = im.n_frames - 1
    im.seek(last)
    # test1: the whole last frame (sender pane left, receiver tcpdump right)
    im.convert("RGB").save(os.path.join(outdir, "test1_last.png"))
    # test2: the last sender line of every 8th frame from 96 on
    strip("test2.gif", range(96, 233, 8), (160, 440, 260, 480), os.path.join(outdir, "test2_ports.png"))
    print("wrote", outdir)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/gif_ports")
