# bucket streams: J = 4 then J = 3 on the keying stream, J = 2 on the second
# side stream (the batch's stream only waits); A/B against the product's
# J = 4 / keying stream, J = 3 / second side stream, J = 2 / batch stream
EDITS = [
    ("sg_kernels.hip", "            js[1] = side[1].s;\n", "            js[0] = side[1].s;\n"),
]
