'use strict';
// TEST INFRASTRUCTURE ONLY (golden-fixture generation).
//
// Restatement of the few PlayCanvas engine math routines the reference's hot
// path calls.  The reference pins npm `playcanvas@2.11.8`
// (/root/reference/package-lock.json:4186-4189); the package is not installed
// in this image and cannot be fetched, so its published algorithms are
// restated here with the engine's evaluation order:
//   Quat.setFromEulerAngles / mul2 / normalize / length   (src/core/math/quat.js)
//   Mat3.setFromQuat                                      (src/core/math/mat3.js)
//   Mat4.setTRS / transformPoint                          (src/core/math/mat4.js)
// Mat3 / Mat4 keep their entries in Float32Array storage, exactly as the
// engine does; Quat / Vec3 components are JS numbers (f64).
// Call sites in the reference: process.ts:71-83, transform.ts:13-14,29,36,
// compressed-chunk.ts:129.

const DEG_TO_RAD = Math.PI / 180;

class Vec3 {
    constructor(x = 0, y = 0, z = 0) {
        this.x = x; this.y = y; this.z = z;
    }

    set(x, y, z) {
        this.x = x; this.y = y; this.z = z;
        return this;
    }
}
Vec3.ZERO = Object.freeze(new Vec3(0, 0, 0));

class Quat {
    constructor(x = 0, y = 0, z = 0, w = 1) {
        this.x = x; this.y = y; this.z = z; this.w = w;
    }

    set(x, y, z, w) {
        this.x = x; this.y = y; this.z = z; this.w = w;
        return this;
    }

    length() {
        return Math.sqrt(this.x * this.x + this.y * this.y + this.z * this.z + this.w * this.w);
    }

    normalize(src = this) {
        let len = src.length();
        if (len === 0) {
            this.x = this.y = this.z = 0;
            this.w = 1;
        } else {
            len = 1 / len;
            this.x = src.x * len;
            this.y = src.y * len;
            this.z = src.z * len;
            this.w = src.w * len;
        }
        return this;
    }

    mul2(lhs, rhs) {
        const q1x = lhs.x, q1y = lhs.y, q1z = lhs.z, q1w = lhs.w;
        const q2x = rhs.x, q2y = rhs.y, q2z = rhs.z, q2w = rhs.w;
        this.x = q1w * q2x + q1x * q2w + q1y * q2z - q1z * q2y;
        this.y = q1w * q2y + q1y * q2w + q1z * q2x - q1x * q2z;
        this.z = q1w * q2z + q1z * q2w + q1x * q2y - q1y * q2x;
        this.w = q1w * q2w - q1x * q2x - q1y * q2y - q1z * q2z;
        return this;
    }

    setFromEulerAngles(ex, ey, ez) {
        const halfToRad = 0.5 * DEG_TO_RAD;
        ex *= halfToRad;
        ey *= halfToRad;
        ez *= halfToRad;
        const sx = Math.sin(ex), cx = Math.cos(ex);
        const sy = Math.sin(ey), cy = Math.cos(ey);
        const sz = Math.sin(ez), cz = Math.cos(ez);
        this.x = sx * cy * cz - cx * sy * sz;
        this.y = cx * sy * cz + sx * cy * sz;
        this.z = cx * cy * sz - sx * sy * cz;
        this.w = cx * cy * cz + sx * sy * sz;
        return this;
    }
}
Quat.IDENTITY = Object.freeze(new Quat(0, 0, 0, 1));

const quatProducts = (r) => {
    const qx = r.x, qy = r.y, qz = r.z, qw = r.w;
    const x2 = qx + qx, y2 = qy + qy, z2 = qz + qz;
    return {
        xx: qx * x2, xy: qx * y2, xz: qx * z2,
        yy: qy * y2, yz: qy * z2, zz: qz * z2,
        wx: qw * x2, wy: qw * y2, wz: qw * z2
    };
};

class Mat3 {
    constructor() {
        this.data = new Float32Array([1, 0, 0, 0, 1, 0, 0, 0, 1]);
    }

    setFromQuat(r) {
        const p = quatProducts(r);
        const m = this.data;
        m[0] = (1 - (p.yy + p.zz));
        m[1] = (p.xy + p.wz);
        m[2] = (p.xz - p.wy);
        m[3] = (p.xy - p.wz);
        m[4] = (1 - (p.xx + p.zz));
        m[5] = (p.yz + p.wx);
        m[6] = (p.xz + p.wy);
        m[7] = (p.yz - p.wx);
        m[8] = (1 - (p.xx + p.yy));
        return this;
    }
}

class Mat4 {
    constructor() {
        this.data = new Float32Array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]);
    }

    setTRS(t, r, s) {
        const p = quatProducts(r);
        const sx = s.x, sy = s.y, sz = s.z;
        const m = this.data;
        m[0] = (1 - (p.yy + p.zz)) * sx;
        m[1] = (p.xy + p.wz) * sx;
        m[2] = (p.xz - p.wy) * sx;
        m[3] = 0;
        m[4] = (p.xy - p.wz) * sy;
        m[5] = (1 - (p.xx + p.zz)) * sy;
        m[6] = (p.yz + p.wx) * sy;
        m[7] = 0;
        m[8] = (p.xz + p.wy) * sz;
        m[9] = (p.yz - p.wx) * sz;
        m[10] = (1 - (p.xx + p.yy)) * sz;
        m[11] = 0;
        m[12] = t.x;
        m[13] = t.y;
        m[14] = t.z;
        m[15] = 1;
        return this;
    }

    transformPoint(vec, res = new Vec3()) {
        const m = this.data;
        const x = vec.x, y = vec.y, z = vec.z;
        res.x = x * m[0] + y * m[4] + z * m[8] + m[12];
        res.y = x * m[1] + y * m[5] + z * m[9] + m[13];
        res.z = x * m[2] + y * m[6] + z * m[10] + m[14];
        return res;
    }
}

module.exports = { Vec3, Quat, Mat3, Mat4, DEG_TO_RAD };
